"""Same-box A/B of the attention kernels at the cfg-2 shape WITH dropout
(p = 0.01, the bench's setting): times relattn_fwd and relattn_bwd with HIP
events (median of N launches) for the library MSQ_LIB_PATH points at, and
saves dqkv / dR / out so a second run can compare against it.
Usage: python tools/attn_abx.py <tag> <out_dir> [ref_tag]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

_pkgload.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from midiseq import attention, ops  # noqa: E402

tag, odir = sys.argv[1], sys.argv[2]
ref = sys.argv[3] if len(sys.argv) > 3 else None
dev = "cuda"
B, T, d, H = int(os.environ.get("MB_B", 32)), 2048, 1024, 8
S = T + 6
p = float(os.environ.get("MB_P", 0.01))
g = torch.Generator(device=dev).manual_seed(0)
bf = torch.bfloat16
qkv = (torch.randn(B * S, 3 * d, device=dev, generator=g) * 0.5).to(bf)
R = (torch.randn(H, S, 128, device=dev, generator=g) * 0.5).to(bf)
dout = torch.randn(B * S, d, device=dev, generator=g).to(bf)
drop = None
if p > 0:
    masks = ops.dropout_attn_mask(B, H, S, 1234, 777, p, dev)
    drop = (masks, p)
scale = d ** -0.5
out, lse = attention.relattn_fwd(qkv, R, B, S, H, 128, scale, drop=drop)
dqkv = torch.empty_like(qkv)
dR = torch.zeros(H, S, 128, device=dev)


def med(fn, n=7):
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return sorted(ts)[n // 2], min(ts)


fwd = med(lambda: attention.relattn_fwd(qkv, R, B, S, H, 128, scale, out=out, lse=lse, drop=drop))
bwd = med(lambda: attention.relattn_bwd(dout, out, lse, qkv, R, B, S, H, 128, scale, dqkv=dqkv, dR=dR, drop=drop))
dR.zero_()
attention.relattn_bwd(dout, out, lse, qkv, R, B, S, H, 128, scale, dqkv=dqkv, dR=dR, drop=drop)
torch.cuda.synchronize()
line = f"{tag}: fwd {fwd[0]:.3f} (min {fwd[1]:.3f}) ms  bwd {bwd[0]:.3f} (min {bwd[1]:.3f}) ms"
os.makedirs(odir, exist_ok=True)
np.savez(os.path.join(odir, f"{tag}.npz"), dqkv=dqkv[:S].float().cpu().numpy(), dR=dR.cpu().numpy(),
         out=out[:S].float().cpu().numpy())
if ref and os.path.exists(os.path.join(odir, f"{ref}.npz")):
    r = np.load(os.path.join(odir, f"{ref}.npz"))
    for k, v in (("dqkv", dqkv[:S].float().cpu().numpy()), ("dR", dR.cpu().numpy()),
                 ("out", out[:S].float().cpu().numpy())):
        den = np.abs(r[k]).max() + 1e-30
        line += f"  {k} maxdiff/max {np.abs(v - r[k]).max() / den:.2e}"
print(line, flush=True)
