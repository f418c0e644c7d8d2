"""Worker of tests/test_ddp_gpu.py (not a test module): one rank of a
world-2 data-parallel step on the ONE leased GPU, process group gloo over
CUDA tensors, through the real TrainStep: forward, fused filtered CE, the
two-stream backward with the engine's per-layer bucket hooks (ddp.GradBuckets
all-reducing on its side stream), fused Adam with the 1/world scale.
Rank 0 writes the averaged gradient and the updated parameters to an .npz.

Mode "rccl1" (world 1, backend nccl = RCCL, through setup_distributed()):
TrainStep(ddp=True) keeps the bucket path at world size 1, so every layer
bucket is a real ProcessGroupNCCL all_reduce issued from the side stream,
waited on that stream (h.wait()), with the per-bucket Adam after it.

usage (under torch.distributed.run): ddp_worker.py <transformer|mamba> <same|split|bucketcheck|rccl1> <out.npz>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import _pkgload  # noqa: E402

_pkgload.load()
from midiseq.train_parallel import TrainStep, setup_distributed  # noqa: E402


def build_model(kind):
    """Small bf16 configs on the MFMA paths (hs = 128 attention)."""
    if kind == "transformer":
        from midiseq.transformer import Transformer, TransformerConfig
        return Transformer(TransformerConfig(n_embd=256, n_heads=2, n_layer=2, block_len=128, dropout=0.0))
    from midiseq.mamba import Mamba
    return Mamba(d_model=256, n_layers=2)


def full_batch(T=128, B=4):
    from oracle.fill import REAL, grammar_tokens
    rng = np.random.default_rng(21)
    w = np.stack([grammar_tokens(rng, REAL, T + 1) for _ in range(B)])
    meta = np.array([[519, 279, 202, 202, 202, 178], [432, 277, 202, 202, 202, 173],
                     [437, 279, 272, 202, 202, 180], [452, 272, 202, 202, 202, 184]][:B])
    return torch.from_numpy(w[:, :-1].copy()), torch.from_numpy(w[:, 1:].copy()), torch.from_numpy(meta)


def rank_slice(mode, rank, world, B=4):
    if mode == "same":
        return slice(0, B // world)
    # "split" and "bucketcheck": each rank its own rows
    n = B // world
    return slice(rank * n, (rank + 1) * n)


class _CallLog:
    """libmidiseq launch observer (midiseq._lib.TAP): keeps the last calls so
    that a failing rank names the launches before its error (a device fault
    surfaces at a later API call; AMD_SERIALIZE_KERNEL=3 makes it the next one)."""

    def __init__(self, n=12):
        self.names, self.n = [], n

    path = os.environ.get("MSQ_TRACE_CALLS")  # diagnostics: a file; synchronise after every launch

    def __call__(self, name, args, launch):
        self.names = (self.names + [name])[-self.n:]
        if self.path:
            with open(f"{self.path}.{os.environ.get('RANK')}", "a") as f:
                f.write(name + " " + " ".join(str(getattr(x, "value", x)) for x in args[:12]) + "\n")
        r = launch()
        if self.path:
            torch.cuda.synchronize()
            with open(f"{self.path}.{os.environ.get('RANK')}", "a") as f:
                f.write("  ok\n")
        return r


def main():
    from midiseq import _lib
    log = _CallLog()
    _lib.TAP = log
    try:
        _main()
    except BaseException:
        print(f"rank {os.environ.get('RANK')}: last libmidiseq calls {log.names}", file=sys.stderr, flush=True)
        raise


def _main():
    kind, mode, out = sys.argv[1], sys.argv[2], sys.argv[3]
    if mode == "rccl1":
        return _main_rccl1(kind, out)
    rank, _, world = setup_distributed(backend="gloo")
    assert world == 2
    torch.cuda.set_device(0)
    model = build_model(kind).to("cuda")
    if rank == 1:  # the parameter broadcast of TrainStep (DDP ctor) must overwrite this
        with torch.no_grad():
            model.flat.data.mul_(1.5)
    step = TrainStep(model)
    assert step.buckets is not None
    flat0 = model.flat.data.clone()  # after the parameter broadcast
    src, trg, meta = full_batch()
    sl = rank_slice(mode, rank, world)
    loss = step(src[sl].cuda(), trg[sl].cuda(), meta[sl].cuda())
    torch.cuda.synchronize()
    extra = {}
    if mode == "bucketcheck":
        # the same step's reduced gradients through one global fused Adam (the
        # MSQ_GLOBAL_ADAM=1 update) from the same start: the per-bucket Adam
        # inside the backward must have produced these parameters bit for bit
        from midiseq import ops
        ref = flat0.clone()
        m, v = torch.zeros_like(ref), torch.zeros_like(ref)
        ops.adam_step(ref, step.grads, m, v, step.step_no, step.lr, step.betas[0], step.betas[1], step.eps,
                      grad_scale=1.0 / world)
        torch.cuda.synchronize()
        extra = dict(ref=ref.cpu().numpy(), m=step.m.cpu().numpy(), m_ref=m.cpu().numpy(), v=step.v.cpu().numpy(),
                     v_ref=v.cpu().numpy())
    if rank == 0:
        np.savez(out, grads=(step.grads / world).cpu().numpy(), flat=model.flat.data.cpu().numpy(),
                 loss=loss.item(), **extra)
    dist.barrier()
    dist.destroy_process_group()


def _main_rccl1(kind, out):
    """World 1 over RCCL: the bucketed step (two steps, so the second runs on
    Adam moments the per-bucket updates wrote) against one global fused Adam
    over the same reduced gradients (bitwise), and the step's gradients
    against a non-DDP TrainStep from the same start."""
    from midiseq import ops
    rank, local, world = setup_distributed()
    assert world == 1 and dist.get_backend() == "nccl", (world, dist.get_backend())
    torch.manual_seed(0)
    model = build_model(kind).to(torch.device("cuda", local))
    start = model.flat.data.clone()
    # the mamba case takes the bucket path from MSQ_DDP_BUCKETS=1 (set by the
    # test: bench.py under torch.distributed.run with one rank), the
    # transformer case from the argument
    step = TrainStep(model, ddp=None if os.environ.get("MSQ_DDP_BUCKETS") == "1" else True)
    assert step.buckets is not None and step.buckets.force and step.eng.layer_grad_ready is not None
    src, trg, meta = (t[0:2].cuda() for t in full_batch())
    ref, m, v = model.flat.data.clone(), torch.zeros_like(start), torch.zeros_like(start)
    for _ in range(2):
        loss = step(src, trg, meta)
        torch.cuda.synchronize()
        # the same reduced gradients through one global Adam from the same start
        ops.adam_step(ref, step.grads, m, v, step.step_no, step.lr, step.betas[0], step.betas[1], step.eps)
        torch.cuda.synchronize()
    g_ddp = step.grads.cpu().numpy()
    flat_ddp, ref_np = model.flat.data.cpu().numpy(), ref.cpu().numpy()
    m_ddp, v_ddp = step.m.cpu().numpy(), step.v.cpu().numpy()
    # a plain (bucket-free) TrainStep, two steps from the same start
    model2 = build_model(kind).to(torch.device("cuda", local))
    with torch.no_grad():
        model2.flat.data.copy_(start)
    plain = TrainStep(model2, ddp=False)
    assert plain.buckets is None
    for _ in range(2):
        loss2 = plain(src, trg, meta)
    torch.cuda.synchronize()
    np.savez(out, grads=g_ddp, grads_plain=plain.grads.cpu().numpy(), flat=flat_ddp, ref=ref_np,
             flat_plain=model2.flat.data.cpu().numpy(), m=m_ddp, m_ref=m.cpu().numpy(), v=v_ddp,
             v_ref=v.cpu().numpy(), loss=loss.item(), loss_plain=loss2.item(), backend=dist.get_backend())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
