"""Why the lm_head forward runs slower than the other forward shapes: the
persistent tile on lm-like shapes with the epilogue, N and the C row pitch
varied one at a time (random bf16 operands), torch.matmul beside each.
Usage: python tools/gemm_lm.py"""
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


dev, bf = "cuda", torch.bfloat16
K = 1024
for M, N, ldc, epi, name in [(65536, 17914, 17920, L.EPI_BIAS, "lm bias"),
                             (65536, 17914, 17920, L.EPI_NONE, "lm none"),
                             (65536, 17920, 18432, L.EPI_NONE, "lm ldc18432"),
                             (65536, 16384, 16384, L.EPI_NONE, "N16384"),
                             (65536, 16384, 16896, L.EPI_NONE, "N16384 ldc16896"),
                             (65536, 4096, 4096, L.EPI_NONE, "N4096"),
                             (65536, 4096, 4608, L.EPI_NONE, "N4096 ldc4608"),
                             (16384, 17914, 17920, L.EPI_NONE, "lm M16384")]:
    A = torch.randn(M, K, device=dev).to(bf)
    W = torch.randn((N + 7) // 8 * 8, K, device=dev).to(bf)[:N]
    C = torch.empty(M, ldc, device=dev, dtype=bf)[:, :N]
    bias = torch.randn(N, device=dev) if epi == L.EPI_BIAS else None
    t = timeit(lambda: ops.gemm(A, W, out=C, epilogue=epi, bias=bias))
    Ct = torch.empty(M, N, device=dev, dtype=bf)
    tt = timeit(lambda: torch.matmul(A, W.t(), out=Ct))
    fl = 2.0 * M * N * K
    print(f"{name:18s} {M}x{N}x{K} ldc {ldc}: msq {t:.3f} ms {fl / t / 1e9:6.0f} TF   torch {tt:.3f} ms "
          f"{fl / tt / 1e9:6.0f} TF", flush=True)
