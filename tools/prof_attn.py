"""Runs the cfg-2 attention fwd+bwd a few times (for rocprofv3 --stats)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload
_pkgload.load()
import torch
from midiseq import attention
dev = "cuda"
B, T, d, H = int(os.environ.get("MB_B", 32)), 2048, 1024, 8
S = T + 6
bf = torch.bfloat16
qkv = (torch.randn(B * S, 3 * d, device=dev) * 0.5).to(bf)
R = (torch.randn(H, S, 128, device=dev) * 0.5).to(bf)
out, lse = attention.relattn_fwd(qkv, R, B, S, H, 128, d ** -0.5)
dout = torch.randn(B * S, d, device=dev).to(bf)
dqkv = torch.empty_like(qkv)
dR = torch.zeros(H, S, 128, device=dev)
for _ in range(3):
    attention.relattn_fwd(qkv, R, B, S, H, 128, d ** -0.5, out=out, lse=lse)
    attention.relattn_bwd(dout, out, lse, qkv, R, B, S, H, 128, d ** -0.5, dqkv=dqkv, dR=dR)
torch.cuda.synchronize()
print("done")
