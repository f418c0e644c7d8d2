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
hp = dict(n_embd=128, n_heads=8, n_layer=2, block_len=64)
cfg = TransformerConfig(vocab_size=REAL.size, metadata_vocab_size=568, precision="fp32", **hp)
shapes = otr.param_shapes(hp["n_embd"], hp["n_heads"], hp["n_layer"], hp["block_len"], REAL.size, 568)
p = {k: v.requires_grad_(True) for k, v in otr.filled_params(shapes).items()}
m = Transformer(cfg).to(dev)
m.load_state_dict({k: v.detach() for k, v in p.items()})
rng = np.random.default_rng(0)
w = np.stack([grammar_tokens(rng, REAL, 65) for _ in range(2)])
src, trg = torch.from_numpy(w[:, :-1].copy()), torch.from_numpy(w[:, 1:].copy())
meta = torch.tensor([[519, 279, 202, 202, 202, 178], [432, 277, 202, 202, 202, 173]])
logits = m(src.cuda(), meta.cuda())
loss = filtered_cross_entropy(src.cuda(), logits, trg.cuda())
loss.backward()
rl = otr.forward(p, src, meta, 2, 8)
oloss.loss(src, trg, rl, REAL).backward()
g = m.grad_dict()
for k in ["blocks.0.sa.heads.0.rel_pos_emb", "blocks.1.sa.heads.3.rel_pos_emb", "blocks.0.sa.heads.0.query.weight"]:
    a, r = g[k].cpu().double(), p[k].grad.double()
    print(k, "normrel", ((a - r).norm() / r.norm()).item())
    if a.dim() == 2 and "rel_pos" in k:
        e = (a - r).norm(dim=1) / (r.norm(dim=1) + 1e-30)
        top = torch.argsort(e, descending=True)[:8]
        for t in top.tolist():
            print("  row", t, "rel", e[t].item(), "refnorm", r[t].norm().item(), "gotnorm", a[t].norm().item())
