"""Persistent 256-tile GEMM on chosen shapes vs torch.matmul (hipBLASLt), random
bf16 operands, HIP-event timing. Usage: python tools/gemm_shapes.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

_pkgload.load()
import torch  # noqa: E402

from midiseq import ops  # noqa: E402
from midiseq import _lib as L  # noqa: E402


def timeit(fn, iters=20, warm=5):
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


g = torch.Generator(device="cuda").manual_seed(0)
bf = torch.bfloat16
shapes = [(65536, 17920, 1024, "lm"), (65536, 3072, 1024, "qkv"), (65536, 4096, 1024, "ffn1"),
          (65536, 1024, 4096, "ffn2"), (65536, 1024, 1024, "proj"), (16384, 17920, 1024, "lm/4"),
          (65536, 8192, 1024, "N8k"), (65536, 17920, 4096, "lmK4k")]
for M, N, K, name in shapes:
    x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(bf)
    w = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(bf)
    y = torch.empty(M, N, device="cuda", dtype=bf)
    bias = torch.randn(N, device="cuda", generator=g)
    fl = 2.0 * M * N * K
    t0 = timeit(lambda: ops.gemm(x, w, out=y))
    t1 = timeit(lambda: ops.gemm(x, w, out=y, epilogue=L.EPI_BIAS, bias=bias))
    t2 = timeit(lambda: torch.matmul(x, w.t(), out=y))
    print(f"{name:6s} {M}x{N}x{K}: none {t0:.3f} ms {fl / t0 / 1e9:.0f} TF  bias {t1:.3f} ms {fl / t1 / 1e9:.0f} TF  "
          f"blas {t2:.3f} ms {fl / t2 / 1e9:.0f} TF", flush=True)
    del x, w, y
