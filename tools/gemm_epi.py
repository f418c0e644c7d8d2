"""What each fused epilogue of the persistent tile costs: the cfg-2 products
with their train-step epilogue against the same product with none (random
operands, HIP events, median of rounds). Usage: python tools/gemm_epi.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

_pkgload.load()
import torch  # noqa: E402

from midiseq import ops  # noqa: E402
from midiseq import _lib as L  # noqa: E402


def timeit(fn, iters=20, warm=4):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


dev, bf, f32 = "cuda", torch.bfloat16, torch.float32
M, d = 32 * 2054, 1024
r = lambda *s, dt=bf: torch.randn(*s, device=dev).to(dt)  # noqa: E731
x1, x4 = r(M, d), r(M, 4 * d)
w1, w4, w44 = r(4 * d, d), r(d, 4 * d), r(4 * d, d)
wt1 = r(d, d)
bias1, bias4 = torch.randn(d, device=dev), torch.randn(4 * d, device=dev)
res = torch.randn(M, d, device=dev)
o1f, o1b, o4b = torch.empty(M, d, device=dev), torch.empty(M, d, device=dev, dtype=bf), torch.empty(M, 4 * d, device=dev, dtype=bf)
hmask = r(M, 4 * d)
db4 = torch.zeros(4 * d, device=dev)
cases = [
    ("ffn1 fwd  none", lambda: ops.gemm(x1, w44, out=o4b)),
    ("ffn1 fwd  bias+relu", lambda: ops.gemm(x1, w44, out=o4b, epilogue=L.EPI_BIAS_RELU, bias=bias4)),
    ("ffn2 dX   none (tb)", lambda: ops.gemm(x1, w4, tb=True, out=o4b)),
    ("ffn2 dX   relu-mask", lambda: ops.gemm(x1, w4, tb=True, out=o4b, epilogue=L.EPI_RELU_MASK, aux=hmask)),
    ("ffn2 dX   relu-mask+colsum", lambda: ops.gemm_colsum(x1, w4, o4b, db4, tb=True, epilogue=L.EPI_RELU_MASK, aux=hmask)),
    ("ffn2 fwd  none f32", lambda: ops.gemm(x4, w4, out=o1f)),
    ("ffn2 fwd  bias+resid f32", lambda: ops.gemm(x4, w4, out=o1f, epilogue=L.EPI_BIAS_RESID, bias=bias1, aux=res)),
    ("ffn2 fwd  bias+drop+resid f32", lambda: ops.gemm(x4, w4, out=o1f, epilogue=L.EPI_BIAS_RESID, bias=bias1, aux=res, drop=(7, 3, 0.01))),
    ("proj fwd  none f32", lambda: ops.gemm(x1, wt1, out=o1f)),
    ("proj fwd  bias+drop+resid f32", lambda: ops.gemm(x1, wt1, out=o1f, epilogue=L.EPI_BIAS_RESID, bias=bias1, aux=res, drop=(7, 3, 0.01))),
    ("proj dX   none bf16", lambda: ops.gemm(x1, wt1, out=o1b)),
]
for rnd in range(2):
    for name, fn in cases:
        t = timeit(fn)
        print(f"{rnd} {name:32s} {t:.3f} ms", flush=True)
