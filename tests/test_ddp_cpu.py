"""Multi-process (gloo, world_size 2, CPU) check of the data-parallel gradient
exchange used by the MI355X train step (ddp.GradBuckets over the flat
gradient layout): averaging the two ranks' bucketed all-reduced gradients
equals the single-process gradient of the concatenated batch (the loss is a
mean over B*T with equal per-rank batches). Per-rank gradients come from the
CPU oracle (the GPU engine is exercised by the gpu tests)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import loss as oloss
from oracle import transformer as otr
from oracle.fill import TINY, grammar_tokens

HP = dict(n_embd=32, n_heads=4, n_layer=2, block_len=16)
MV = 10


def _batch():
    rng = np.random.default_rng(5)
    w = np.stack([grammar_tokens(rng, TINY, 17) for _ in range(4)])
    meta = rng.integers(0, MV, size=(4, 6))
    return torch.from_numpy(w[:, :-1].copy()), torch.from_numpy(w[:, 1:].copy()), torch.from_numpy(meta)


def _grads(src, trg, meta):
    shapes = otr.param_shapes(HP["n_embd"], HP["n_heads"], HP["n_layer"], HP["block_len"], TINY.size, MV)
    p = {k: v.requires_grad_(True) for k, v in otr.filled_params(shapes).items()}
    oloss.loss(src, trg, otr.forward(p, src, meta, HP["n_layer"], HP["n_heads"]), TINY).backward()
    return {k: v.grad for k, v in p.items()}


def _flat(grads):
    import _pkgload
    _pkgload.load()
    from midiseq.transformer import TransformerConfig, ParamLayout, reference_keys, _select
    cfg = TransformerConfig(vocab_size=TINY.size, metadata_vocab_size=MV, precision="fp32", **HP)
    lay = ParamLayout(cfg)
    flat = torch.zeros(lay.numel)
    V = lay.views(flat)
    for k, (name, sel) in reference_keys(cfg).items():
        if name != "__tril__":
            _select(V[name], sel).copy_(grads[k])
    return flat, lay


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import _pkgload
    _pkgload.load()
    from midiseq.ddp import GradBuckets, transformer_buckets
    src, trg, meta = _batch()
    sl = slice(rank * 2, rank * 2 + 2)
    flat, lay = _flat(_grads(src[sl], trg[sl], meta[sl]))
    # per-bucket update as TrainStep runs it (on_reduced after each bucket's
    # SUM): an elementwise step over the reduced slice; it must see every
    # bucket exactly once, after its reduction, with the 1/world scale
    param = torch.zeros_like(flat)
    seen = []

    def update(s, e, scale):
        seen.append((s, e))
        param[s:e] -= 0.5 * flat[s:e] * scale

    gb = GradBuckets(flat, transformer_buckets(lay), on_reduced=update)
    # same notification order as the backward engine: head, layers L-1..0, embeddings
    for key in ["head"] + list(reversed(range(HP["n_layer"]))) + [-1]:
        gb.ready(key)
    scale = gb.finish()
    assert not gb.uncovered() and sorted(seen) == sorted(gb.ranges.values())
    if rank == 0:
        q.put(((flat * scale).numpy(), (-2.0 * param).numpy()))
    dist.destroy_process_group()


def test_two_rank_average_equals_full_batch():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, upd = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    src, trg, meta = _batch()
    full, lay = _flat(_grads(src, trg, meta))
    np.testing.assert_allclose(got, full.numpy(), rtol=1e-4, atol=1e-7)
    np.testing.assert_array_equal(upd, got)  # the per-bucket update saw the averaged gradient


def test_bucket_ranges_cover_layout_exactly():
    import _pkgload
    _pkgload.load()
    from midiseq.transformer import TransformerConfig, ParamLayout
    from midiseq.ddp import transformer_buckets
    lay = ParamLayout(TransformerConfig())
    r = sorted(transformer_buckets(lay).values())
    assert r[0][0] == 0 and r[-1][1] == lay.numel
    for (a, b), (c, d) in zip(r, r[1:]):
        assert b == c
