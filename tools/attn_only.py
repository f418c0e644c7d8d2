"""Runs the relative-attention forward (and optionally backward) at the cfg-2
shape a few times: a small target for rocprofv3 PMC passes.
Usage: python tools/attn_only.py [fwd|bwd|both] [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

_pkgload.load()
import torch  # noqa: E402

from midiseq import attention  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "fwd"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
B, T, d, H = 32, 2048, 1024, 8
S = T + 6
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
qkv = (torch.randn(B * S, 3 * d, device=dev, generator=g) * 0.5).bfloat16()
R = (torch.randn(H, S, 128, device=dev, generator=g) * 0.5).bfloat16()
scale = d ** -0.5
out, lse = attention.relattn_fwd(qkv, R, B, S, H, 128, scale)
dout = torch.randn(B * S, d, device=dev, generator=g).bfloat16()
dqkv = torch.empty_like(qkv)
dR = torch.zeros(H, S, 128, device=dev)
for _ in range(iters):
    if which in ("fwd", "both"):
        attention.relattn_fwd(qkv, R, B, S, H, 128, scale, out=out, lse=lse)
    if which in ("bwd", "both"):
        attention.relattn_bwd(dout, out, lse, qkv, R, B, S, H, 128, scale, dqkv=dqkv, dR=dR)
torch.cuda.synchronize()
print("done")
