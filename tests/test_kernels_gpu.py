"""GPU parity of the building-block kernels against torch fp32 CPU references.

Tolerances: fp32 path (exact mode) 1e-5 relative; bf16 path uses bf16-rounded
inputs and fp32 accumulation, compared against an fp32 product of the SAME
rounded inputs at 2e-3 relative (accumulation order only)."""
import pytest
import torch

from midiseq import ops
from midiseq import _lib as L

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 1), (1, 0)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(256, 384, 128), (130, 70, 72), (64, 17914 // 32 * 8 + 2, 64)])
def test_gemm_layouts(ta, tb, dtype, M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N + K)
    a = torch.randn(M, K, generator=g).to(dtype)
    b = torch.randn(N, K, generator=g).to(dtype)
    ref = a.float() @ b.float().t()
    A = (a.t().contiguous() if ta else a).to(dev)
    Bm = (b.t().contiguous() if tb else b).to(dev)
    if (ta and M % 8) or (tb and N % 8):
        pytest.skip("bf16/ld alignment needs ld % 8 == 0")
    out = ops.gemm(A, Bm, ta=bool(ta), tb=bool(tb), out_dtype=torch.float32)
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    assert _rel(out, ref) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogues(dtype):
    g = torch.Generator().manual_seed(3)
    M, N, K = 200, 256, 192
    a = torch.randn(M, K, generator=g).to(dtype)
    w = torch.randn(N, K, generator=g).to(dtype)
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    base = a.float() @ w.float().t()
    A, W, bi, R = a.to(dev), w.to(dev), bias.to(dev), res.to(dev)
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    o = ops.gemm(A, W, out_dtype=torch.float32, epilogue=L.EPI_BIAS, bias=bi)
    assert _rel(o, base + bias) < tol
    o = ops.gemm(A, W, out_dtype=torch.float32, epilogue=L.EPI_BIAS_RELU, bias=bi)
    assert _rel(o, torch.relu(base + bias)) < tol
    o = ops.gemm(A, W, out_dtype=torch.float32, epilogue=L.EPI_BIAS_RESID, bias=bi, aux=R)
    assert _rel(o, base + bias + res) < tol
    o = ops.gemm(A, W, out_dtype=torch.float32, epilogue=L.EPI_RELU_MASK, aux=R)
    assert _rel(o, base * (res > 0)) < tol
    acc = R.clone()
    ops.gemm(A, W, out=acc, epilogue=L.EPI_ACCUM)
    assert _rel(acc, base + res) < tol
    ob = ops.gemm(A, W, out_dtype=torch.bfloat16, epilogue=L.EPI_BIAS, bias=bi)
    assert _rel(ob.float(), base + bias) < 1e-2


@pytest.mark.parametrize("M,N,K", [(3000, 4096, 1024), (65728 // 8, 1024, 512), (100, 256, 64)])
@pytest.mark.parametrize("epi", ["relu_mask", "none"])
def test_gemm_colsum_bias_grad(M, N, K, epi):
    """msq_gemm_colsum: the FFN dX product (dY . W) with the column sums of its
    bf16 output fused into the 256 tile's epilogue (fp32 sums before rounding,
    fixed-order reduction; small shapes: msq_gemm_ex + msq_colsum), with and
    without accumulation into the bias gradient."""
    g = torch.Generator().manual_seed(M + N + K)
    dy = torch.randn(M, K, generator=g).bfloat16()
    w = torch.randn(K, N, generator=g).bfloat16()  # [K][N]: tb
    h = torch.randn(M, N, generator=g).bfloat16()
    base = dy.float() @ w.float()
    if epi == "relu_mask":
        base = base * (h.float() > 0)
    Dy, Wd, Hd = dy.to(dev), w.to(dev), h.to(dev)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    db = torch.full((N,), 0.5, device=dev)
    e = L.EPI_RELU_MASK if epi == "relu_mask" else L.EPI_NONE
    ops.gemm_colsum(Dy, Wd, out, db, tb=True, epilogue=e, aux=Hd if epi == "relu_mask" else None, accumulate=True)
    torch.cuda.synchronize()
    assert _rel(out.float(), base) < 1e-2
    # fused: fp32 sums before rounding; the small-shape fallback sums the bf16 C
    tol = 2e-3 if M >= 256 else 1e-2
    assert _rel(db - 0.5, base.sum(0)) < tol
    db2 = torch.empty(N, device=dev)
    ops.gemm_colsum(Dy, Wd, out, db2, tb=True, epilogue=e, aux=Hd if epi == "relu_mask" else None)
    torch.cuda.synchronize()
    assert torch.equal(db2, db - 0.5) or _rel(db2, base.sum(0)) < tol
    db3 = torch.empty(N, device=dev)  # bitwise reproducible (no atomics)
    ops.gemm_colsum(Dy, Wd, out, db3, tb=True, epilogue=e, aux=Hd if epi == "relu_mask" else None)
    torch.cuda.synchronize()
    assert torch.equal(db2, db3)


@pytest.mark.parametrize("M", [1, 5, 16, 33, 64])
@pytest.mark.parametrize("N,K", [(17, 64), (1024, 1032), (4384, 1024), (1024, 2048), (1024, 4096), (1020, 3000),
                                 (1022, 4096)])
def test_gemm_skinny_decode_shapes(M, N, K):
    """M <= 64 rows (decode steps) take the weight-streaming kernel
    (gemm_skinny.hip): row / column / K edges and every forward epilogue,
    A with a padded leading dimension, fp32 and bf16 outputs; N 1024 / 1020
    at K 4096 / 3000 split K over workgroups (fp32 partials in the ops.gemm
    workspace + skinny_reduce_kernel), N 1022 (N % 4 != 0) does not."""
    g = torch.Generator().manual_seed(M * 31 + N + K)
    a = torch.randn(M, K, generator=g).bfloat16()
    w = torch.randn(N, K, generator=g).bfloat16()
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    base = a.float() @ w.float().t()
    A = torch.zeros(M, K + 8, device=dev, dtype=torch.bfloat16)[:, :K]  # lda = K + 8
    A.copy_(a)
    W, bi, R = w.to(dev), bias.to(dev), res.to(dev)
    assert A.stride(0) == K + 8
    assert _rel(ops.gemm(A, W, out_dtype=torch.float32), base) < 2e-3
    assert _rel(ops.gemm(A, W, out_dtype=torch.float32, epilogue=L.EPI_BIAS, bias=bi), base + bias) < 2e-3
    assert _rel(ops.gemm(A, W, out_dtype=torch.float32, epilogue=L.EPI_BIAS_RELU, bias=bi),
                torch.relu(base + bias)) < 2e-3
    assert _rel(ops.gemm(A, W, out_dtype=torch.float32, epilogue=L.EPI_BIAS_RESID, bias=bi, aux=R),
                base + bias + res) < 2e-3
    ob = ops.gemm(A, W, out_dtype=torch.bfloat16, epilogue=L.EPI_BIAS, bias=bi)
    assert _rel(ob.float(), base + bias) < 1e-2


ROUTES = {"persistent": L.ROUTE_DEFAULT, "tile256": L.ROUTE_TILE256, "tile128": L.ROUTE_TILE128}


@pytest.mark.parametrize("route", list(ROUTES))
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 1), (1, 0)])
@pytest.mark.parametrize("M,N,K", [(4104, 2056, 1000), (2304, 4096, 512), (1800, 776, 64)])
def test_gemm256_layouts_and_edges(route, ta, tb, M, N, K):
    """Large products on each kernel family (msq_gemm_set_route): the
    persistent 256 tile (forward / dX products), the per-tile 256 LDS-DMA tile
    and the 128 tile; M/N/K edges are zero-filled by the buffer descriptor
    (K % 64 != 0, M % 256 != 0, a single K-step), fp32 and bf16 outputs."""
    g = torch.Generator().manual_seed(M + N + K + ta + 2 * tb)
    a = torch.randn(M, K, generator=g).bfloat16()
    b = torch.randn(N, K, generator=g).bfloat16()
    ref = a.float() @ b.float().t()
    A = (a.t().contiguous() if ta else a).to(dev)
    Bm = (b.t().contiguous() if tb else b).to(dev)
    with ops.gemm_route(ROUTES[route]):
        out = ops.gemm(A, Bm, ta=bool(ta), tb=bool(tb), out_dtype=torch.float32)
        outb = ops.gemm(A, Bm, ta=bool(ta), tb=bool(tb), out_dtype=torch.bfloat16)
        torch.cuda.synchronize()
        assert _rel(out, ref) < 2e-3
        assert _rel(outb.float(), ref) < 1e-2
        acc = torch.randn(M, N, generator=g).to(dev)
        ref2 = acc.cpu() + ref
        ops.gemm(A, Bm, ta=bool(ta), tb=bool(tb), out=acc, epilogue=L.EPI_ACCUM)
        assert _rel(acc, ref2) < 2e-3


def test_gemm256_splitk_weight_grad():
    """dW = dY^T X with K = tokens (split-K over 16 slices, fp32 atomics)."""
    g = torch.Generator().manual_seed(11)
    Kt, M, N = 32776, 1024, 1024
    dy = (torch.randn(Kt, M, generator=g) * 0.1).bfloat16()
    x = torch.randn(Kt, N, generator=g).bfloat16()
    ref = dy.float().t() @ x.float()
    G = torch.full((M, N), 0.5, device=dev)
    ops.gemm(dy.to(dev), x.to(dev), ta=True, tb=True, out=G, epilogue=L.EPI_ACCUM)
    assert _rel(G.cpu() - 0.5, ref) < 2e-3


@pytest.mark.parametrize("route", list(ROUTES))
@pytest.mark.parametrize("M", [3000, 4096])
def test_gemm256_epilogues_bf16_out(route, M):
    """Every forward / dX epilogue on each kernel family, with and without an
    M tail (3000 = 11 x 256 + 184)."""
    g = torch.Generator().manual_seed(12 + M)
    N, K = 3072, 1024
    a = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    base = a.float() @ w.float().t()
    A, W, bi, R = a.to(dev), w.to(dev), bias.to(dev), res.to(dev)
    with ops.gemm_route(ROUTES[route]):
        o = ops.gemm(A, W, out_dtype=torch.bfloat16)
        assert _rel(o.float(), base) < 1e-2
        o = ops.gemm(A, W, out_dtype=torch.bfloat16, epilogue=L.EPI_BIAS, bias=bi)
        assert _rel(o.float(), base + bias) < 1e-2
        o = ops.gemm(A, W, out_dtype=torch.bfloat16, epilogue=L.EPI_BIAS_RELU, bias=bi)
        assert _rel(o.float(), torch.relu(base + bias)) < 1e-2
        o = ops.gemm(A, W, out_dtype=torch.float32, epilogue=L.EPI_BIAS_RESID, bias=bi, aux=R)
        assert _rel(o, base + bias + res) < 2e-3
        o = ops.gemm(A, W, out_dtype=torch.bfloat16, epilogue=L.EPI_RELU_MASK, aux=R.bfloat16())
        assert _rel(o.float(), base * (res.bfloat16().float() > 0)) < 1e-2
        o = ops.gemm(A, W, out_dtype=torch.float32, epilogue=L.EPI_RELU_MASK, aux=R)
        assert _rel(o, base * (res > 0)) < 2e-3
        # dropout + residual epilogue: the same keep mask on every route
        o = ops.gemm(A, W, out_dtype=torch.float32, epilogue=L.EPI_BIAS_RESID, bias=bi, aux=R, drop=(7, 3, 0.1))
        kept = (o.cpu() - res) != 0
        frac = kept.float().mean().item()
        assert 0.88 < frac < 0.92, frac
        assert _rel(torch.where(kept, o.cpu(), torch.zeros(())), torch.where(kept, (base + bias) / 0.9 + res,
                                                                             torch.zeros(()))) < 2e-3


def _pack_bits(h):
    """MSQ_MASK1 reference: word [m][w] bit c = (h[m][32 w + c] > 0), as int32"""
    M, N = h.shape
    nw = (N + 31) // 32
    pos = torch.zeros(M, nw * 32, dtype=torch.int64)
    pos[:, :N] = (h.float().cpu() > 0).long()
    words = (pos.view(M, nw, 32) << torch.arange(32)).sum(-1)
    return ((words + 2 ** 31) % 2 ** 32 - 2 ** 31).int()


@pytest.mark.parametrize("route", list(ROUTES))
@pytest.mark.parametrize("M,N,K", [(3000, 4096, 1024), (65728 // 16, 1024, 256), (100, 512, 64)])
def test_gemm_relu_bits(route, M, N, K):
    """MSQ_MASK1: the FFN1 forward (BIAS_RELU) writes the 1-bit ReLU mask of
    its stored bf16 output (in the persistent tile's epilogue, else one pass
    over C) and the FFN2 dX product reads it (RELU_MASK, plain and with the
    fused bias column sums): the mask is exact, C is unchanged, and the dX
    outputs equal those masked by the bf16 activation itself, bitwise."""
    g = torch.Generator().manual_seed(M + N + K + len(route))
    a = torch.randn(M, K, generator=g).bfloat16().to(dev)
    w = (torch.randn(N, K, generator=g) * 0.05).bfloat16().to(dev)
    bias = torch.randn(N, generator=g).to(dev)
    dy = torch.randn(M, K, generator=g).bfloat16().to(dev)
    w2 = torch.randn(K, N, generator=g).bfloat16().to(dev)  # [K][N]: tb
    with ops.gemm_route(ROUTES[route]):
        h0 = ops.gemm(a, w, out_dtype=torch.bfloat16, epilogue=L.EPI_BIAS_RELU, bias=bias)
        bits = torch.full((M, (N + 31) // 32 + 2), -7, device=dev, dtype=torch.int32)[:, :(N + 31) // 32]
        h = ops.gemm(a, w, out_dtype=torch.bfloat16, epilogue=L.EPI_BIAS_RELU, bias=bias, aux=bits)
        torch.cuda.synchronize()
        assert torch.equal(h, h0)
        assert torch.equal(bits.cpu(), _pack_bits(h))
        o_ref = ops.gemm(dy, w2, tb=True, out_dtype=torch.bfloat16, epilogue=L.EPI_RELU_MASK, aux=h)
        o = ops.gemm(dy, w2, tb=True, out_dtype=torch.bfloat16, epilogue=L.EPI_RELU_MASK, aux=bits)
        torch.cuda.synchronize()
        assert torch.equal(o, o_ref)
        out_ref, out = torch.empty_like(o), torch.empty_like(o)
        db_ref, db = torch.zeros(N, device=dev), torch.zeros(N, device=dev)
        ops.gemm_colsum(dy, w2, out_ref, db_ref, tb=True, epilogue=L.EPI_RELU_MASK, aux=h)
        ops.gemm_colsum(dy, w2, out, db, tb=True, epilogue=L.EPI_RELU_MASK, aux=bits)
        torch.cuda.synchronize()
        assert torch.equal(out, out_ref)
        # below the 256 tile's size (and on the 128 tile's route) the columns are
        # summed by msq_colsum, whose split rows add in a varying order
        assert torch.equal(db, db_ref) or _rel(db, db_ref) < 1e-5


def test_gemm_routes_bitwise_mask_and_layout():
    """The persistent tile's bf16 store widening (16-lane swaps) against the
    per-tile kernel: identical bf16 outputs, bitwise, on a shape with several
    tiles per workgroup (M tail, 2 K-steps)."""
    g = torch.Generator().manual_seed(3)
    M, N, K = 2 * 256 * 256 + 40, 512, 128
    a = torch.randn(M, K, generator=g).bfloat16().to(dev)
    w = torch.randn(N, K, generator=g).bfloat16().to(dev)
    with ops.gemm_route(L.ROUTE_DEFAULT):
        p = ops.gemm(a, w, out_dtype=torch.bfloat16)
    with ops.gemm_route(L.ROUTE_TILE256):
        q = ops.gemm(a, w, out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    assert torch.equal(p, q)


def test_gemm_batched_strided():
    g = torch.Generator().manual_seed(5)
    Bt, S, T, d, V = 3, 70, 64, 128, 200
    x = torch.randn(Bt, S, d, generator=g).bfloat16()
    w = torch.randn(V, d, generator=g).bfloat16()
    ref = (x[:, S - T:].float() @ w.float().t())
    X = x.to(dev)
    out = torch.empty(Bt, T, V + 8, device=dev)[:, :, :V]
    ops.gemm(X[:, S - T:], w.to(dev), out=out)
    assert _rel(out, ref) < 2e-3


@pytest.mark.parametrize("d", [32, 128, 1024, 1500, 2048])
@pytest.mark.parametrize("ydt", [torch.float32, torch.bfloat16])
def test_layernorm(d, ydt):
    g = torch.Generator().manual_seed(d)
    rows = 333
    x = torch.randn(rows, d, generator=g) * 3 + 1
    gamma = torch.randn(d, generator=g)
    beta = torch.randn(d, generator=g)
    dy = torch.randn(rows, d, generator=g)
    xr = x.clone().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    yref = torch.nn.functional.layer_norm(xr, (d,), gr, br, 1e-5)
    yref.backward(dy)
    y, mean, rstd = ops.layernorm_fwd(x.to(dev), gamma.to(dev), beta.to(dev), out_dtype=ydt)
    assert _rel(y.float(), yref.detach()) < (1e-5 if ydt == torch.float32 else 1e-2)
    acc = torch.ones(rows, d, device=dev)
    dg = torch.zeros(d, device=dev)
    db = torch.zeros(d, device=dev)
    cp = torch.empty(rows, d, device=dev, dtype=torch.bfloat16)
    ops.layernorm_bwd(acc, dy.to(dev), x.to(dev), mean, rstd, gamma.to(dev), dg, db, dx_copy=cp, ordered=False)
    assert _rel(acc - 1, xr.grad) < 1e-5
    assert _rel(dg, gr.grad) < 1e-5 and _rel(db, br.grad) < 1e-5
    assert _rel(cp.float(), acc) < 1e-2
    # the fixed-order schedule (the default) against the same reference, and
    # bitwise equal from one launch to the next
    outs = []
    for _ in range(2):
        acc2 = torch.ones(rows, d, device=dev)
        dg2, db2, dbias2 = (torch.zeros(d, device=dev) for _ in range(3))
        ops.layernorm_bwd(acc2, dy.to(dev), x.to(dev), mean, rstd, gamma.to(dev), dg2, db2, dbias=dbias2, ordered=True)
        outs.append((acc2, dg2, db2, dbias2))
    acc2, dg2, db2, dbias2 = outs[0]
    assert _rel(acc2 - 1, xr.grad) < 1e-5
    assert _rel(dg2, gr.grad) < 1e-5 and _rel(db2, br.grad) < 1e-5
    assert _rel(dbias2, acc2.sum(0).cpu()) < 1e-5
    assert all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))


def test_embedding():
    g = torch.Generator().manual_seed(1)
    V, MV, d, B, T = 50, 9, 64, 3, 17
    tok = torch.randn(V, d, generator=g)
    met = torch.randn(MV, d, generator=g)
    idx = torch.randint(0, V, (B, T), generator=g)
    meta = torch.randint(0, MV, (B, 6), generator=g)
    ref = torch.cat([met[meta], tok[idx]], dim=1)
    x = torch.empty(B, T + 6, d, device=dev)
    ops.embed_fwd(x, tok.to(dev), met.to(dev), idx.to(dev), meta.to(dev))
    assert torch.equal(x.cpu(), ref)
    dx = torch.randn(B, T + 6, d, generator=g)
    gt = torch.zeros(V, d, device=dev)
    gm = torch.zeros(MV, d, device=dev)
    ops.embed_bwd(gt, gm, dx.to(dev), idx.to(dev), meta.to(dev), deterministic=False)
    rt = torch.zeros(V, d).index_add_(0, idx.reshape(-1), dx[:, 6:].reshape(-1, d))
    rm = torch.zeros(MV, d).index_add_(0, meta.reshape(-1), dx[:, :6].reshape(-1, d))
    assert _rel(gt, rt) < 1e-5 and _rel(gm, rm) < 1e-5


def _embed_bwd_seq(V, MV, idx, meta, dx):
    """fp64 scatter-add in sequence order (the order the sorted path sums in)."""
    d = dx.shape[-1]
    nm = meta.shape[1]
    rt = torch.zeros(V, d, dtype=torch.float64)
    rm = torch.zeros(MV, d, dtype=torch.float64)
    rt.index_add_(0, idx.reshape(-1), dx[:, nm:].reshape(-1, d).double())
    rm.index_add_(0, meta.reshape(-1), dx[:, :nm].reshape(-1, d).double())
    return rt, rm


@pytest.mark.parametrize("case", ["small", "skewed", "ragged_d", "one_hot_key", "large"])
def test_embedding_sorted_deterministic(case):
    """msq_embed_bwd_sorted: same sums as the fp64 scatter-add and bitwise equal
    across repeats (the atomic path is not). 'skewed': one token id holds half
    the rows, so its sorted run spans many 64-row blocks (partials + fix pass);
    'one_hot_key': every row the same id; 'large': cfg-2 vocabularies and width (two radix passes)."""
    g = torch.Generator().manual_seed(11)
    V, MV, d, B, T, nm = {"small": (50, 9, 64, 3, 17, 6), "skewed": (300, 20, 256, 4, 700, 6),
                          "ragged_d": (37, 5, 516, 2, 333, 3), "one_hot_key": (10, 4, 128, 3, 500, 2),
                          "large": (17914, 568, 1024, 4, 2048, 6)}[case]
    idx = torch.randint(0, V, (B, T), generator=g)
    meta = torch.randint(0, MV, (B, nm), generator=g)
    if case == "skewed":
        hot = torch.rand(B, T, generator=g) < 0.5
        idx[hot] = 7
    if case == "one_hot_key":
        idx.fill_(3)
        meta.fill_(1)
    dx = torch.randn(B, T + nm, d, generator=g)
    outs = []
    for _ in range(2):
        gt = torch.full((V, d), 0.5, device=dev)  # accumulates into what is there
        gm = torch.full((MV, d), -0.25, device=dev)
        ops.embed_bwd(gt, gm, dx.to(dev), idx.to(dev), meta.to(dev))
        outs.append((gt.cpu(), gm.cpu()))
    rt, rm = _embed_bwd_seq(V, MV, idx, meta, dx)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert (outs[0][0].double() - 0.5 - rt).abs().max() <= 1e-5 * (1 + rt.abs().max())
    assert (outs[0][1].double() + 0.25 - rm).abs().max() <= 1e-5 * (1 + rm.abs().max())


def test_embedding_sorted_drops_out_of_range_ids():
    g = torch.Generator().manual_seed(12)
    V, MV, d, B, T, nm = 20, 6, 64, 2, 90, 3
    idx = torch.randint(0, V, (B, T), generator=g)
    meta = torch.randint(0, MV, (B, nm), generator=g)
    idx[0, :5] = V + 3
    idx[1, 7] = -1
    meta[1, 0] = MV
    dx = torch.randn(B, T + nm, d, generator=g)
    gt = torch.zeros(V, d, device=dev)
    gm = torch.zeros(MV, d, device=dev)
    ops.embed_bwd(gt, gm, dx.to(dev), idx.to(dev), meta.to(dev))
    ok_t = (idx >= 0) & (idx < V)
    ok_m = meta < MV
    rt = torch.zeros(V, d).index_add_(0, idx[ok_t], dx[:, nm:][ok_t])
    rm = torch.zeros(MV, d).index_add_(0, meta[ok_m], dx[:, :nm][ok_m])
    assert _rel(gt, rt) < 1e-5 and _rel(gm, rm) < 1e-5


def test_colsum_and_cast():
    g = torch.Generator().manual_seed(2)
    x = torch.randn(1000, 300, generator=g)
    out = torch.zeros(300, device=dev)
    ops.colsum(x.to(dev), out)
    assert _rel(out, x.sum(0)) < 1e-5
    xb = torch.empty(1000, 300, device=dev, dtype=torch.bfloat16)
    ops.cast(xb, x.to(dev))
    assert torch.equal(xb.cpu(), x.bfloat16())


def test_adam_matches_torch():
    g = torch.Generator().manual_seed(4)
    n = 10007
    p0 = torch.randn(n, generator=g)
    p = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([p], lr=5e-5)
    P, M, Vv = p0.clone().to(dev), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    sh = torch.empty(n, device=dev, dtype=torch.bfloat16)
    for step in range(1, 4):
        gr = torch.randn(n, generator=g)
        p.grad = gr.clone()
        opt.step()
        ops.adam_step(P, gr.to(dev), M, Vv, step, 5e-5, shadow=sh)
    assert _rel(P, p.detach()) < 1e-6
    assert torch.equal(sh.cpu(), P.cpu().bfloat16())


@pytest.mark.parametrize("route", list(ROUTES))
def test_gemm_resid_epilogues_bf16_aux(route):
    """BIAS_RESID / BIAS_DROP_RESID with a bf16 residual (aux_dtype MSQ_BF16)
    on every kernel family, M with a tail (3000 = 11 x 256 + 184): the aux is
    read as bf16 everywhere (it was read as fp32 outside the skinny kernel:
    wrong columns, and past the end of the buffer on the last rows)."""
    from oracle import dropout as odrop
    g = torch.Generator().manual_seed(31)
    M, N, K = 3000, 1024, 512
    a = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g).bfloat16()
    base = a.float() @ w.float().t() + bias
    A, W, bi, R = a.to(dev), w.to(dev), bias.to(dev), res.to(dev)
    with ops.gemm_route(ROUTES[route]):
        o = ops.gemm(A, W, out_dtype=torch.float32, epilogue=L.EPI_BIAS_RESID, bias=bi, aux=R)
        assert _rel(o, base + res.float()) < 2e-3
        ob = ops.gemm(A, W, out_dtype=torch.bfloat16, epilogue=L.EPI_BIAS_RESID, bias=bi, aux=R)
        assert _rel(ob.float(), base + res.float()) < 1e-2
        seed, site, p = 5, 9, 0.2
        o = ops.gemm(A, W, out_dtype=torch.float32, epilogue=L.EPI_BIAS_RESID, bias=bi, aux=R, drop=(seed, site, p))
        keep = torch.from_numpy(odrop.keep(seed, site, M, N, p))
        ref = res.float() + torch.where(keep, base * odrop.scale(p), torch.zeros(()))
        assert _rel(o, ref) < 2e-3


@pytest.mark.parametrize("epi", ["drop", "relu_mask", "none"])
def test_gemm256_tail_rows_split(epi):
    """M = 64*256 + 100 rows, N = 1024: the 256 tile runs rows [0, 16384) and
    the 128 tile the 100 tail rows (msq_gemm_ex wave-quantisation split); the
    dropout hash must stay keyed by the GLOBAL row."""
    from oracle import dropout as odrop
    g = torch.Generator().manual_seed(21)
    M, N, K = 64 * 256 + 100, 1024, 128
    a = torch.randn(M, K, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * 0.1).bfloat16()
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    base = a.float() @ w.float().t()
    A, W = a.to(dev), w.to(dev)
    if epi == "drop":
        seed, site, p = 77, 3, 0.2
        o = ops.gemm(A, W, out_dtype=torch.float32, epilogue=L.EPI_BIAS_RESID, bias=bias.to(dev), aux=res.to(dev),
                     drop=(seed, site, p))
        keep = torch.from_numpy(odrop.keep(seed, site, M, N, p))
        ref = res + torch.where(keep, (base + bias) * odrop.scale(p), torch.zeros(()))
        assert _rel(o, ref) < 2e-3
    elif epi == "relu_mask":
        o = ops.gemm(A, W, out_dtype=torch.bfloat16, epilogue=L.EPI_RELU_MASK, aux=res.bfloat16().to(dev))
        assert _rel(o.float(), base * (res.bfloat16().float() > 0)) < 1e-2
    else:
        o = ops.gemm(A, W, out_dtype=torch.float32)
        assert _rel(o, base) < 2e-3


@pytest.mark.parametrize("rows,cols,lds,ldd", [(4256, 1024, 1024, 4256), (1024, 2048, 2048, 1024),
                                               (17914, 1024, 1024, 17920), (70, 130, 136, 72), (33, 45, 47, 35)])
def test_transpose_bf16(rows, cols, lds, ldd):
    """msq_transpose_bf16 (the backward's transposed weight shadows): 16-B
    vector path for aligned rows, element path at ragged edges / odd strides."""
    from midiseq._lib import call, ptr
    g = torch.Generator(device=dev).manual_seed(rows + cols)
    src = torch.randn(rows, lds, device=dev, generator=g).bfloat16()
    dst = torch.full((cols, ldd), 7.0, device=dev, dtype=torch.bfloat16)
    call("msq_transpose_bf16", ptr(dst), ldd, ptr(src), lds, rows, cols, ops.stream())
    torch.cuda.synchronize()
    assert torch.equal(dst[:, :rows], src[:, :cols].t())
    assert bool((dst[:, rows:] == 7.0).all())  # nothing written past the rows


def test_gemm_resid_ln_unfused_rejects_row_pitch():
    """The unfused path of msq_gemm_resid_ln (fp32 operands) normalises C with
    msq_layernorm_fwd, which reads C densely: a padded ldc (or ldy) is
    rejected before anything is written."""
    M, N, K = 8, 256, 64
    g = torch.Generator().manual_seed(5)
    a = torch.randn(M, K, generator=g).to(dev)
    w = torch.randn(N, K, generator=g).to(dev)
    bias, gamma, beta = (torch.randn(N, generator=g).to(dev) for _ in range(3))
    res = torch.randn(M, N, generator=g).to(dev)
    big = torch.full((M, N + 64), 7.0, device=dev)
    y = torch.full((M, N), 7.0, device=dev)
    with pytest.raises(RuntimeError, match="ldc == N"):
        ops.gemm_resid_ln(a, w, big[:, :N], bias, res, gamma, beta, y)
    bigy = torch.full((M, N + 64), 7.0, device=dev)
    c = torch.full((M, N), 7.0, device=dev)
    with pytest.raises(RuntimeError, match="ldy == N"):
        ops.gemm_resid_ln(a, w, c, bias, res, gamma, beta, bigy[:, :N])
    torch.cuda.synchronize()
    assert bool((big == 7.0).all()) and bool((y == 7.0).all())
    assert bool((bigy == 7.0).all()) and bool((c == 7.0).all())


@pytest.mark.parametrize("M", [1, 7, 33, 64])
@pytest.mark.parametrize("N,K", [(1024, 1024), (1024, 4096), (1000, 520), (256, 1024)])
def test_gemm_resid_ln_matches_unfused(M, N, K):
    """msq_gemm_resid_ln (the decode step's residual product with the next
    LayerNorm in its split-K reduce) against msq_gemm (BIAS_RESID) +
    msq_layernorm_fwd: the residual rows equal within fp32 summation order
    (bitwise where both split K the same way), the normalised rows within bf16
    rounding; and the fp32 operand path (which runs the unfused pair) exactly."""
    g = torch.Generator().manual_seed(M * 13 + N + K)
    a = torch.randn(M, K, generator=g).bfloat16().to(dev)
    w = (torch.randn(N, K, generator=g) * 0.05).bfloat16().to(dev)
    bias = torch.randn(N, generator=g).to(dev)
    res = (torch.randn(M, N, generator=g) * 2 + 0.3).to(dev)
    gamma, beta = (1 + 0.1 * torch.randn(N, generator=g)).to(dev), (0.1 * torch.randn(N, generator=g)).to(dev)
    c_ref = ops.gemm(a, w, out_dtype=torch.float32, epilogue=L.EPI_BIAS_RESID, bias=bias, aux=res)
    y_ref = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.layernorm_fwd(c_ref, gamma, beta, out=y_ref)
    c = torch.full((M, N), float("nan"), device=dev)
    y = torch.full((M, N), float("nan"), device=dev).bfloat16()
    ops.gemm_resid_ln(a, w, c, bias, res, gamma, beta, y)
    torch.cuda.synchronize()
    assert _rel(c, c_ref) < 1e-5
    if K > 1024 and K % 512 == 0:
        assert torch.equal(c, c_ref)  # the same K slices and summation order
    assert _rel(y.float(), y_ref.float()) < 1e-2
    # fp32 operands: the unfused pair itself
    af, wf = a.float(), w.float()
    c32, y32 = torch.empty(M, N, device=dev), torch.empty(M, N, device=dev)
    ops.gemm_resid_ln(af, wf, c32, bias, res, gamma, beta, y32)
    c32r = ops.gemm(af, wf, out_dtype=torch.float32, epilogue=L.EPI_BIAS_RESID, bias=bias, aux=res)
    y32r, _, _ = ops.layernorm_fwd(c32r, gamma, beta)
    torch.cuda.synchronize()
    assert torch.equal(c32, c32r) and torch.equal(y32, y32r)
