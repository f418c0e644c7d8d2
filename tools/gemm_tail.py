"""The cfg-2 products whose 256-tile grid leaves a partial last round
(M = 32 x 2054 = 65 728 rows: 1 028 tiles at N = 1 024), through ops.gemm with
the train step's epilogues, HIP-event timing, for the library MSQ_LIB_PATH
points at; saves the outputs so a second run can compare.
Usage: python tools/gemm_tail.py <tag> <out_dir> [ref_tag]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

_pkgload.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from midiseq import ops  # noqa: E402
from midiseq import _lib as L  # noqa: E402

tag, odir = sys.argv[1], sys.argv[2]
ref = sys.argv[3] if len(sys.argv) > 3 else None
g = torch.Generator(device="cuda").manual_seed(0)
bf = torch.bfloat16
M = 32 * 2054
line, outs = [tag], {}
for name, N, K, epi in [("ffn2_fwd", 1024, 4096, "drop"), ("ffn1_dX", 1024, 4096, "none"),
                        ("qkv_dX", 1024, 3072, "none"), ("lm_dX", 1024, 17920, "none"),
                        ("proj_fwd", 1024, 1024, "drop")]:
    x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(bf)
    w = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(bf)  # [N, K]
    y = torch.empty(M, N, device="cuda", dtype=bf)
    if epi == "drop":
        bias = torch.randn(N, device="cuda", generator=g)
        res = torch.randn(M, N, device="cuda", generator=g).to(bf)
        fn = lambda: ops.gemm(x, w, out=y, epilogue=L.EPI_BIAS_RESID, bias=bias, aux=res, drop=(7, 3, 0.01))
    else:
        fn = lambda: ops.gemm(x, w, out=y)
    for _ in range(3):
        fn()
    ts = []
    for _ in range(9):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    line.append(f"{name} {sorted(ts)[4] * 1e3:.0f}us")
    outs[name] = y.float().cpu().numpy()
    del x, w, y
os.makedirs(odir, exist_ok=True)
np.savez(os.path.join(odir, f"{tag}.npz"), **outs)
if ref:
    r = np.load(os.path.join(odir, f"{ref}.npz"))
    for k in outs:
        d = np.abs(outs[k] - r[k])
        line.append(f"{k} maxdiff {d.max():.3g} rows {np.unique(np.nonzero(d)[0])[[0, -1]] if d.any() else '-'}")
print("  ".join(line), flush=True)
