"""Weight-gradient shapes of the cfg-2 step (C += A^T B over K = 65 728 tokens)
in the layout the backward has (both operands token-major: ta = tb = 1, fragments
through ds_read_b64_tr_b16) against the same products with K-contiguous copies
of the operands (ta = 0, tb = 0), and the cost of making those copies
(msq_transpose_bf16). HIP-event timing, random bf16 operands.
Usage: python tools/gemm_dw_layout.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

_pkgload.load()
import torch  # noqa: E402

from midiseq import ops  # noqa: E402
from midiseq import _lib as L  # noqa: E402
from midiseq._lib import ptr, call, stream  # noqa: E402


def timeit(fn, iters=10, warm=3):
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


def main():
    dev = "cuda"
    K, d = 32 * 2054, 1024
    bf = torch.bfloat16
    for name, m, n in (("w2 dW", d, 4 * d), ("w1 dW", 4 * d, d), ("qkv dW", 3 * d, d), ("proj dW", d, d)):
        dy = torch.randn(K, m, device=dev).to(bf)   # token-major gradient rows
        x = torch.randn(K, n, device=dev).to(bf)    # token-major activation rows
        out = torch.zeros(m, n, device=dev)
        fl = 2.0 * m * n * K
        t_tt = timeit(lambda: ops.gemm(dy, x, ta=True, tb=True, out=out, epilogue=L.EPI_ACCUM))
        dyt = torch.empty(m, K, device=dev, dtype=bf)
        xt = torch.empty(n, K, device=dev, dtype=bf)

        def tr():
            call("msq_transpose_bf16", ptr(dyt), K, ptr(dy), m, K, m, stream())
            call("msq_transpose_bf16", ptr(xt), K, ptr(x), n, K, n, stream())
        t_tr = timeit(tr)
        tr()
        out2 = torch.zeros(m, n, device=dev)
        t_nn = timeit(lambda: ops.gemm(dyt, xt, out=out2, epilogue=L.EPI_ACCUM))
        out.zero_()
        out2.zero_()
        ops.gemm(dy, x, ta=True, tb=True, out=out, epilogue=L.EPI_ACCUM)
        ops.gemm(dyt, xt, out=out2, epilogue=L.EPI_ACCUM)
        torch.cuda.synchronize()
        rel = ((out - out2).abs().max() / out.abs().max()).item()
        print(f"{name} {m}x{n}x{K}: TT {t_tt:.3f} ms {fl / t_tt / 1e9:.0f} TF/s | NN {t_nn:.3f} ms "
              f"{fl / t_nn / 1e9:.0f} TF/s | transposes {t_tr:.3f} ms | rel {rel:.1e}", flush=True)


if __name__ == "__main__":
    main()
