"""The cfg-2 train step's LayerNorm backward (ln2 / ln1 shape: rows = 32 x 2054,
d = 1024, bf16 dy, fp32 x, bf16 branch-gradient copy with the dropout mask,
fused bias column sums) launched alone a few times: a small target for
rocprofv3 kernel summaries and PMC passes.
Usage: python tools/ln_only.py [queue|ordered] [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

_pkgload.load()
import torch  # noqa: E402

from midiseq import ops  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "queue"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = "cuda"
B, T, d = 32, 2048, 1024
S = T + 6
rows = B * S
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(rows, d, device=dev, generator=g)
gamma = torch.randn(d, device=dev, generator=g)
beta = torch.randn(d, device=dev, generator=g)
y, mean, rstd = ops.layernorm_fwd(x, gamma, beta, out_dtype=torch.bfloat16)
dy = torch.randn(rows, d, device=dev, generator=g).bfloat16()
acc = torch.zeros(rows, d, device=dev)
cp = torch.empty(rows, d, device=dev, dtype=torch.bfloat16)
dg, db, dbias = (torch.zeros(d, device=dev) for _ in range(3))
for _ in range(iters):
    ops.layernorm_bwd(acc, dy, x, mean, rstd, gamma, dg, db, dx_copy=cp, drop=(1234, 5, 0.01), dbias=dbias,
                      ordered=(mode == "ordered"))
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for _ in range(iters):
    ops.layernorm_bwd(acc, dy, x, mean, rstd, gamma, dg, db, dx_copy=cp, drop=(1234, 5, 0.01), dbias=dbias,
                      ordered=(mode == "ordered"))
ev[1].record()
torch.cuda.synchronize()
print(f"{mode}: {ev[0].elapsed_time(ev[1]) / iters * 1000:.1f} us per launch")
