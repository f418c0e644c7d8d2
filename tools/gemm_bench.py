"""GEMM shapes of the cfg-2 train step: the per-tile 256x256 kernel vs the
default route (persistent tile / split-K) vs torch.matmul (hipBLASLt) as the known-good
reference, random bf16 operands, HIP-event timing on the current stream.
Usage: python tools/gemm_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

_pkgload.load()
import torch  # noqa: E402

from midiseq import ops  # noqa: E402
from midiseq import _lib as L  # noqa: E402


def timeit(fn, iters=30, warm=5):
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
    M, d = 32 * 2054, 1024
    bf = torch.bfloat16
    cases = [
        ("qkv  fwd NT", M, 3 * d, d, 0, 0, L.EPI_NONE),
        ("ffn1 fwd NT +bias+relu", M, 4 * d, d, 0, 0, L.EPI_BIAS_RELU),
        ("ffn2 fwd NT +bias+resid", M, d, 4 * d, 0, 0, L.EPI_BIAS_RESID),
        ("lm   fwd NT +bias", 32 * 2048, 17914, d, 0, 0, L.EPI_BIAS),
        ("ffn2 dX  NN", M, 4 * d, d, 0, 1, L.EPI_RELU_MASK),
        ("ffn1 dX  NN", M, d, 4 * d, 0, 1, L.EPI_NONE),
        ("w2   dW  TT accum", d, 4 * d, M, 1, 1, L.EPI_ACCUM),
        ("w1   dW  TT accum", 4 * d, d, M, 1, 1, L.EPI_ACCUM),
        ("proj dW  TT accum", d, d, M, 1, 1, L.EPI_ACCUM),
        ("lm   dW  TT accum", 17920, d, 32 * 2048, 1, 1, L.EPI_ACCUM),
        ("qkv  dW  TT accum", 3 * d, d, M, 1, 1, L.EPI_ACCUM),
        ("proj fwd NT +bias+resid", M, d, d, 0, 0, L.EPI_BIAS_RESID),
        ("qkv  dX  NN", M, d, 3 * d, 0, 1, L.EPI_NONE),
    ]
    for name, m, n, k, ta, tb, epi in cases:
        pad = lambda r, c: torch.randn(r, (c + 7) // 8 * 8, device=dev).to(bf)[:, :c]  # noqa: E731
        A = pad(k, m) if ta else pad(m, k)
        Bm = pad(k, n) if tb else pad(n, k)
        odt = torch.float32 if epi == L.EPI_ACCUM else bf
        out = torch.zeros(m, (n + 7) // 8 * 8, device=dev, dtype=odt)[:, :n]
        bias = torch.randn(n, device=dev)
        aux = torch.randn(m, n, device=dev).to(bf) if epi == L.EPI_RELU_MASK else (
            torch.randn(m, n, device=dev) if epi == L.EPI_BIAS_RESID else None)
        kw = dict(ta=bool(ta), tb=bool(tb), out=out, epilogue=epi,
                  bias=bias if epi in (L.EPI_BIAS, L.EPI_BIAS_RELU, L.EPI_BIAS_RESID) else None, aux=aux)
        fl = 2.0 * m * n * k
        res = {}
        for tag, route in (("tile256", L.ROUTE_TILE256), ("default", L.ROUTE_DEFAULT)):
            out.zero_()
            with ops.gemm_route(route):
                ms = timeit(lambda: ops.gemm(A, Bm, **kw))
                res[tag] = (ms, fl / ms / 1e9)
                if tag == "default":
                    out.zero_()
                    ops.gemm(A, Bm, **kw)
                    got = out.float()
        At = A.t() if ta else A
        Bt = Bm if tb else Bm.t()
        ms = timeit(lambda: torch.matmul(At, Bt))
        res["torch"] = (ms, fl / ms / 1e9)
        ref = torch.matmul(At.float(), Bt.float()) if m * n <= 4096 * 4096 * 2 else None
        err = ""
        if ref is not None and epi in (L.EPI_NONE, L.EPI_ACCUM):
            err = f" relerr {((got - ref).abs().max() / ref.abs().max()).item():.2e}"
        print(f"{name:26s} " + "  ".join(f"{t} {v[0]:7.3f} ms {v[1]:7.1f} TF" for t, v in res.items()) + err,
              flush=True)


if __name__ == "__main__":
    main()
