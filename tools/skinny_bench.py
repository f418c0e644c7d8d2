"""Times the decode-step skinny products (M = 64 rows) through msq_gemm and
through torch.matmul (hipBLASLt): weight-streaming GB/s per shape.
GPU only:  python tools/skinny_bench.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import _pkgload  # noqa: E402

_pkgload.load()
from midiseq import ops, _lib as L  # noqa: E402


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3  # us


def main():
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = [("mamba in_proj", 64, 4384, 1024, L.EPI_NONE), ("mamba out_proj", 64, 1024, 2048, L.EPI_NONE),
              ("lm_head", 64, 17914, 1024, L.EPI_BIAS), ("tf qkv", 64, 3072, 1024, L.EPI_NONE),
              ("tf ffn1", 64, 4096, 1024, L.EPI_BIAS_RELU), ("tf ffn2", 64, 1024, 4096, L.EPI_BIAS)]
    if len(sys.argv) > 1 and sys.argv[1] == "probe":  # overhead structure of the persistent kernel
        shapes = [("probe m16", 16, 4384, 1024, L.EPI_NONE), ("probe m32", 32, 4384, 1024, L.EPI_NONE),
                  ("probe n256", 64, 256, 1024, L.EPI_NONE), ("probe n4096", 64, 4096, 1024, L.EPI_NONE),
                  ("probe n8192", 64, 8192, 1024, L.EPI_NONE), ("probe n16384", 64, 16384, 1024, L.EPI_NONE),
                  ("probe k512", 64, 4384, 512, L.EPI_NONE)]
    print(f"{'shape':16s} {'M':>3s} {'N':>6s} {'K':>5s} {'msq us':>8s} {'GB/s':>7s} {'blas us':>8s} {'GB/s':>7s}")
    for name, M, N, K, epi in shapes:
        x = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) * 0.02).bfloat16()
        b = torch.randn(N, device=dev, generator=g)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        bias = b if epi != L.EPI_NONE else None
        t_m = timeit(lambda: ops.gemm(x, w, out=y, epilogue=epi, bias=bias))
        t_b = timeit(lambda: torch.matmul(x, w.t()))
        gb = 2.0 * N * K / 1e9
        print(f"{name:16s} {M:3d} {N:6d} {K:5d} {t_m:8.2f} {gb / t_m * 1e6:7.0f} {t_b:8.2f} {gb / t_b * 1e6:7.0f}",
              flush=True)


if __name__ == "__main__":
    main()
