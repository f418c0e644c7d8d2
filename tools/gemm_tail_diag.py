"""A bf16-residual BIAS_RESID product at the cfg-2 FFN2 shape on the default
and tile256 routes, against an fp32 reference (and a second run's outputs).
Usage: python tools/gemm_tail_diag.py <tag> <out_dir>"""
import os, sys
sys.path.insert(0, os.getcwd())
import _pkgload; _pkgload.load()
import numpy as np, torch
from midiseq import ops
from midiseq import _lib as L
tag, odir = sys.argv[1], sys.argv[2]
g = torch.Generator(device="cuda").manual_seed(0)
bf = torch.bfloat16
M, N, K = 32 * 2054, 1024, 4096
x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(bf)
w = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(bf)
bias = torch.randn(N, device="cuda", generator=g)
res = torch.randn(M, N, device="cuda", generator=g).to(bf)
outs = {}
for name, route in [("p0", L.ROUTE_DEFAULT), ("t256", L.ROUTE_TILE256)]:
    y = torch.full((M, N), 7.0, device="cuda", dtype=bf)
    with ops.gemm_route(route):
        ops.gemm(x, w, out=y, epilogue=L.EPI_BIAS_RESID, bias=bias, aux=res)
    torch.cuda.synchronize()
    outs[name] = y.float().cpu().numpy()
ref = (x.float() @ w.float().t() + bias).cpu().numpy() + res.float().cpu().numpy()
os.makedirs(odir, exist_ok=True)
np.savez(os.path.join(odir, tag + ".npz"), **outs)
for k, v in outs.items():
    d = np.abs(v - ref)
    bad = np.nonzero(d.max(1) > 0.5)[0]
    rmax = d.max(1)
    worst = np.argsort(-rmax)[:6]
    big = np.nonzero(rmax > 20)[0]
    print(tag, k, "vs fp32 ref: max", d.max(), "rows > 20:", len(big), big[:6], big[-6:] if len(big) else "", "worst", worst, rmax[worst])
if tag == "B":
    a = np.load(os.path.join(odir, "A.npz"))
    for k in outs:
        d = np.abs(outs[k] - a[k]).max(1)
        nz = np.nonzero(d)[0]
        print("A vs B", k, "rows differing:", len(nz), nz[:8], nz[88:100], nz[-3:] if len(nz) else "")
