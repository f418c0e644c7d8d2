"""A/B of the Mamba SSD paths on the same inputs: bf16 chunk-parallel MFMA path
vs the fp32-LDS sequential kernels (MSQ_MAMBA_SSD_V1=1) vs the fp32 exact
engine; prints loss and per-tensor gradient agreement.
Usage: python tools/mamba_ab.py [d_model] [layers] [T]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

_pkgload.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import mamba2 as om  # noqa: E402
from oracle.fill import REAL, grammar_tokens  # noqa: E402
from midiseq.mamba import Mamba  # noqa: E402
from midiseq.loss import filtered_cross_entropy  # noqa: E402


def run(d, nl, T, precision, v1):
    if v1:
        os.environ["MSQ_MAMBA_SSD_V1"] = "1"
    else:
        os.environ.pop("MSQ_MAMBA_SSD_V1", None)
    m = Mamba(d_model=d, n_layers=nl, precision=precision).to("cuda")
    m.load_state_dict(om.filled_params(om.param_shapes(d, nl, REAL.size, 568)))
    rng = np.random.default_rng(0)
    w = torch.from_numpy(np.stack([grammar_tokens(rng, REAL, T + 1) for _ in range(2)])).cuda()
    meta = torch.tensor([[519, 279, 202, 202, 202, 178], [432, 277, 202, 202, 202, 173]], device="cuda")
    logits = m(w[:, :-1], meta)
    loss = filtered_cross_entropy(w[:, :-1], logits, w[:, 1:])
    loss.backward()
    return loss.item(), {k: v.detach().double().cpu() for k, v in m.grad_dict().items()}


def main():
    d, nl, T = (int(x) for x in (sys.argv[1:] + ["256", "2", "700"])[:3])
    ref = run(d, nl, T, "fp32", False)
    for tag, v1 in (("bf16 v1", True), ("bf16 mfma", False)):
        loss, g = run(d, nl, T, "bf16", v1)
        worst = []
        for k, r in ref[1].items():
            if r.norm() == 0:
                continue
            nr = ((g[k] - r).norm() / r.norm()).item()
            cos = torch.nn.functional.cosine_similarity(g[k].flatten(), r.flatten(), dim=0).item()
            worst.append((nr, cos, k))
        worst.sort(reverse=True)
        print(f"{tag}: loss {loss:.6f} vs fp32 {ref[0]:.6f}; worst grads: " +
              ", ".join(f"{k} nr={nr:.3g} cos={c:.5f}" for nr, c, k in worst[:5]), flush=True)


if __name__ == "__main__":
    main()
