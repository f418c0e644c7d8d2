"""Kernel micro-benchmarks at the cfg-2 shapes (B=32, T=2048, d=1024, h=8).
Times each launch with HIP events on the current stream; prints TFLOP/s."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

_pkgload.load()
import torch  # noqa: E402

from midiseq import ops, attention  # noqa: E402
from midiseq import _lib as L  # noqa: E402


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
    B, T, d, H = int(os.environ.get("MB_B", 32)), 2048, 1024, 8
    S = T + 6
    M = B * S
    bf = torch.bfloat16
    x = torch.randn(M, d, device=dev).to(bf)
    rows = []

    def gemm_case(name, M, N, K, ta, tb):
        A = torch.randn((K, M) if ta else (M, K), device=dev).to(bf)
        Bm = torch.randn((K, N) if tb else (N, K), device=dev).to(bf)
        out = torch.empty(M, N, device=dev, dtype=bf if not (ta and tb) else torch.float32)
        ms = timeit(lambda: ops.gemm(A, Bm, ta=bool(ta), tb=bool(tb), out=out))
        rows.append((name, ms, 2.0 * M * N * K / ms / 1e9))

    gemm_case("qkv  NT 65728x3072x1024", M, 3 * d, d, 0, 0)
    gemm_case("ffn1 NT 65728x4096x1024", M, 4 * d, d, 0, 0)
    gemm_case("ffn2 NT 65728x1024x4096", M, d, 4 * d, 0, 0)
    gemm_case("lm   NT 65536x17920x1024", B * T, 17920, d, 0, 0)
    gemm_case("dX   NN 65728x1024x4096", M, d, 4 * d, 0, 1)
    gemm_case("dW   TN 4096x1024x65728", 4 * d, d, M, 1, 1)
    qkv = (torch.randn(M, 3 * d, device=dev) * 0.5).to(bf)
    R = (torch.randn(H, S, 128, device=dev) * 0.5).to(bf)
    scale = d ** -0.5
    out, lse = attention.relattn_fwd(qkv, R, B, S, H, 128, scale)
    flops_att = 3 * d * S * (S + 1) * B  # causal-useful QK^T, q.R^T, PV
    outs = {}
    for ver in ("1", "2", "3"):
        os.environ["MSQ_ATTN_FWD"] = ver
        ms = timeit(lambda: attention.relattn_fwd(qkv, R, B, S, H, 128, scale, out=out, lse=lse))
        rows.append((f"attn fwd v{ver}", ms, flops_att / ms / 1e9))
        outs[ver] = (out.clone(), lse.clone())
    del os.environ["MSQ_ATTN_FWD"]
    for ver in ("2", "3"):
        print(f"fwd v{ver} vs v1 max abs diff out", (outs[ver][0].float() - outs["1"][0].float()).abs().max().item(),
              "lse", (outs[ver][1] - outs["1"][1]).abs().max().item(), flush=True)
    dout = torch.randn(M, d, device=dev).to(bf)
    dqkv = torch.empty_like(qkv)
    dR = torch.zeros(H, S, 128, device=dev)
    dR.zero_()
    ms = timeit(lambda: attention.relattn_bwd(dout, out, lse, qkv, R, B, S, H, 128, scale, dqkv=dqkv, dR=dR),
                iters=3, warm=1)
    rows.append(("attn bwd", ms, 2 * flops_att / ms / 1e9))
    for n, ms, tf in rows:
        print(f"{n:32s} {ms:9.3f} ms  {tf:8.1f} TFLOP/s")


if __name__ == "__main__":
    main()
