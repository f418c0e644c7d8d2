import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload; _pkgload.load()
import numpy as np, torch
from oracle import loss as oloss, transformer as otr
from oracle.fill import REAL, grammar_tokens
from midiseq.transformer import Transformer, TransformerConfig
from midiseq.loss import filtered_cross_entropy
dev = "cuda"
prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
hp = dict(n_embd=256, n_heads=2, n_layer=2, block_len=128)
cfg = TransformerConfig(vocab_size=REAL.size, metadata_vocab_size=568, precision=prec, **hp)
m = Transformer(cfg).to(dev)
shapes = otr.param_shapes(hp["n_embd"], hp["n_heads"], hp["n_layer"], hp["block_len"], REAL.size, 568)
p = otr.filled_params(shapes)
m.load_state_dict(p)
rng = np.random.default_rng(9)
B, T = 2, 128
w = np.stack([grammar_tokens(rng, REAL, T + 1) for _ in range(B)])
src, trg = torch.from_numpy(w[:, :-1].copy()), torch.from_numpy(w[:, 1:].copy())
meta = torch.tensor([[519, 279, 202, 202, 202, 178], [432, 277, 202, 202, 202, 173]])
logits = m(src.to(dev), meta.to(dev))
loss = filtered_cross_entropy(src.to(dev), logits, trg.to(dev))
loss.backward()
pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
ref_logits = otr.forward(pr, src, meta, hp["n_layer"], hp["n_heads"])
ref_loss = oloss.loss(src, trg, ref_logits, REAL)
ref_loss.backward()
print("loss", loss.item(), ref_loss.item(), "logit err", (logits.detach().float().cpu() - ref_logits.detach()).abs().max().item())
gd = m.grad_dict()
for k in gd:
    ref = pr[k].grad
    g = gd[k].cpu().double().reshape(-1); r = ref.double().reshape(-1)
    e = (g - r).abs().max().item() / (r.abs().max().item() + 1e-12)
    nr = ((g - r).norm() / (r.norm() + 1e-30)).item()
    cos = (g @ r / (g.norm() * r.norm() + 1e-30)).item()
    if e > 1e-2 or "ffwd" in k:
        print(f"{k:45s} maxrel {e:.3e} normrel {nr:.3e} cos {cos:.5f} refmax {r.abs().max().item():.3e}")
