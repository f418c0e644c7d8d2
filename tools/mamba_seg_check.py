"""Diagnostic: segmented vs three-kernel SSD path (MSQ_MAMBA_SSD_3K) vs the fp32
oracle at T = 700 (11 chunks, segments of 3): loss, y and gradient norm-relative errors."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _pkgload  # noqa: E402

_pkgload.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import loss as oloss, mamba2 as om  # noqa: E402
from oracle.fill import REAL, grammar_tokens  # noqa: E402
from test_mamba_gpu import build  # noqa: E402
from midiseq.loss import filtered_cross_entropy  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 700
rng = np.random.default_rng(11)
B = 2
w = np.stack([grammar_tokens(rng, REAL, T + 1) for _ in range(B)])
src, trg = torch.from_numpy(w[:, :-1].copy()), torch.from_numpy(w[:, 1:].copy())
meta = torch.tensor([[519, 279, 202, 202, 202, 178], [432, 277, 202, 202, 202, 173]])
res = {}
for three in (True, False):
    if three:
        os.environ["MSQ_MAMBA_SSD_3K"] = "1"
    else:
        os.environ.pop("MSQ_MAMBA_SSD_3K", None)
    m, p = build(256, 2, "bf16")
    logits = m(src.cuda(), meta.cuda())
    loss = filtered_cross_entropy(src.cuda(), logits, trg.cuda())
    loss.backward()
    res[three] = (loss.item(), logits.detach().float().cpu(), {k: v.detach().cpu().double() for k, v in m.grad_dict().items()})
pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
rl = om.forward(pr, src, meta, 2)
rloss = oloss.loss(src, trg, rl, REAL)
rloss.backward()
print(f"T={T} loss 3K {res[True][0]:.6f} seg {res[False][0]:.6f} oracle {rloss.item():.6f}")
print(f"logits 3K-seg max {float((res[True][1] - res[False][1]).abs().max()):.3e}  oracle-seg max "
      f"{float((rl.detach() - res[False][1]).abs().max()):.3e} oracle-3K {float((rl.detach() - res[True][1]).abs().max()):.3e}")
for k in res[True][2]:
    a, b = res[True][2][k].reshape(-1), res[False][2][k].reshape(-1)
    r = pr[k].grad.double().reshape(-1) if pr[k].grad is not None else None
    if r is None or r.norm() < 1e-12:
        continue
    print(f"{k:40s} 3K-vs-seg nr {((a - b).norm() / a.norm()).item():.2e}  seg-vs-oracle nr {((b - r).norm() / r.norm()).item():.2e}"
          f"  3K-vs-oracle nr {((a - r).norm() / r.norm()).item():.2e}")
