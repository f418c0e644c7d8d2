"""Runs a few cfg-2 GEMM shapes (forward NT, dX NN, dW TT) and the attention
forward a few times each, for rocprofv3 PMC passes (tools/attn_pmc.sh style).
Usage: python tools/prof_gemm.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

_pkgload.load()
import torch  # noqa: E402

from midiseq import ops, attention  # noqa: E402
from midiseq import _lib as L  # noqa: E402

dev = "cuda"
bf = torch.bfloat16
M, d = 32 * 2054, 1024
pad = lambda r, c: torch.randn(r, (c + 7) // 8 * 8, device=dev).to(bf)[:, :c]  # noqa: E731
cases = [("ffn1 fwd", M, 4 * d, d, 0, 0), ("ffn2 dX", M, d, 4 * d, 0, 1), ("w1 dW", 4 * d, d, M, 1, 1)]
for name, m, n, k, ta, tb in cases:
    A = pad(k, m) if ta else pad(m, k)
    Bm = pad(k, n) if tb else pad(n, k)
    epi = L.EPI_ACCUM if ta else L.EPI_NONE
    out = torch.zeros(m, (n + 7) // 8 * 8, device=dev, dtype=torch.float32 if ta else bf)[:, :n]
    for _ in range(3):
        ops.gemm(A, Bm, ta=bool(ta), tb=bool(tb), out=out, epilogue=epi)
B, T, H = 32, 2048, 8
S = T + 6
qkv = (torch.randn(B * S, 3 * d, device=dev) * 0.5).to(bf)
R = (torch.randn(H, S, 128, device=dev) * 0.5).to(bf)
for _ in range(3):
    attention.relattn_fwd(qkv, R, B, S, H, 128, d ** -0.5)
torch.cuda.synchronize()
print("done")
