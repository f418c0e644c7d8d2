"""Times the train step's GEMM shapes (cfg 2: d 1024, FFN 4096, V 17914,
B*S = 32*2054 rows) through msq_gemm and through torch.matmul (hipBLASLt) in
the same storage layouts, to see where the hand-written tiles stand against
the vendor library.  GPU only:  python tools/gemm_vs_blas.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import _pkgload  # noqa: E402

_pkgload.load()
from midiseq import ops, _lib as L  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    dev = "cuda"
    M = 32 * 2054
    shapes = [("qkv", 3072, 1024), ("proj", 1024, 1024), ("ffn1", 4096, 1024), ("ffn2", 1024, 4096), ("lm", 17920, 1024)]
    g = torch.Generator(device=dev).manual_seed(0)
    print(f"{'shape':6s} {'kind':4s} {'msq ms':>8s} {'TF/s':>7s} {'t256 ms':>8s} {'TF/s':>7s} {'blas ms':>8s} {'TF/s':>7s}")
    for name, N, K in shapes:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g) * 0.02
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16, generator=g)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(N, K, device=dev, dtype=torch.float32)
        dwb = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        cases = [
            ("fwd", lambda: ops.gemm(x, w, out=y), lambda: torch.matmul(x, w.t(), out=y)),
            ("dX", lambda: ops.gemm(dy, w, tb=True, out=dx), lambda: torch.matmul(dy, w, out=dx)),
            ("dW", lambda: ops.gemm(dy, x, ta=True, tb=True, out=dw, epilogue=L.EPI_ACCUM),
             lambda: torch.matmul(dy.t(), x, out=dwb)),
        ]
        if name == "ffn2":  # the fused epilogues of the train step on this shape
            h = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
            res = torch.randn(M, N, device=dev, dtype=torch.float32, generator=g)
            bias = torch.randn(N, device=dev, dtype=torch.float32, generator=g)
            yf = torch.empty(M, N, device=dev, dtype=torch.float32)
            cases += [
                ("dXrm", lambda: ops.gemm(dy, w, tb=True, out=dx, epilogue=L.EPI_RELU_MASK, aux=h),
                 lambda: torch.matmul(dy, w, out=dx)),
                ("fwdd", lambda: ops.gemm(x, w, out=yf, epilogue=L.EPI_BIAS_RESID, bias=bias, aux=res,
                                          drop=(1, 2, 0.01)),
                 lambda: torch.matmul(x, w.t(), out=y)),
            ]
        for kind, a, b in cases:
            ta_ = timeit(a)
            with ops.gemm_route(L.ROUTE_TILE256):
                tt_ = timeit(a)
            tb_ = timeit(b)
            print(f"{name:6s} {kind:4s} {ta_:8.3f} {fl / ta_ / 1e9:7.1f} {tt_:8.3f} {fl / tt_ / 1e9:7.1f} "
                  f"{tb_:8.3f} {fl / tb_ / 1e9:7.1f}", flush=True)
        # correctness spot check of fwd against BLAS
        ops.gemm(x, w, out=y)
        ref = torch.matmul(x, w.t())
        err = (y.float() - ref.float()).abs().max().item()
        print(f"       fwd max|diff| vs blas {err:.3e}", flush=True)


if __name__ == "__main__":
    main()
