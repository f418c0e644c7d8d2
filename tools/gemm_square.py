import os, sys, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '.')
import _pkgload; _pkgload.load()
from midiseq import ops
def timeit(fn, n=20):
    for _ in range(3): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize(); return s.elapsed_time(e) / n
g = torch.Generator(device='cuda').manual_seed(0)
for M, N, K in [(4096, 4096, 4096), (8192, 8192, 8192), (65728, 3072, 1024), (65728, 3072, 4096), (65728, 1024, 4096), (16384, 16384, 1024)]:
    if os.environ.get('MSQ_SQ_DATA') == 'randn':
        x = torch.randn(M, K, device='cuda', generator=g).bfloat16()
        w = (torch.randn(N, K, device='cuda', generator=g) * 0.02).bfloat16()
    elif os.environ.get('MSQ_SQ_DATA') == 'zero':
        x = torch.zeros(M, K, device='cuda').bfloat16()
        w = torch.zeros(N, K, device='cuda').bfloat16()
    else:
        x = torch.rand(M, K, device='cuda', generator=g).bfloat16() * 2 - 1
        w = torch.rand(N, K, device='cuda', generator=g).bfloat16() * 2 - 1
    y = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
    t1 = timeit(lambda: ops.gemm(x, w, out=y)); t2 = timeit(lambda: torch.matmul(x, w.t(), out=y))
    fl = 2.0 * M * N * K
    print(f"{os.environ.get('MSQ_SQ_DATA', 'uniform')} {M}x{N}x{K}: msq {t1:.3f} ms {fl/t1/1e9:.0f} TF/s   blas {t2:.3f} ms {fl/t2/1e9:.0f} TF/s", flush=True)
