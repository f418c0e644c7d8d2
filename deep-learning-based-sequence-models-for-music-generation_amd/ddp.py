"""Data-parallel gradient exchange for the flat gradient buffer.

Replaces the implicit collectives of ``DDP(model)`` in train_parallel.py:151:
  * parameters are broadcast from rank 0 ONCE (DDP ctor);
  * the 1.08 GB per-forward buffer broadcast of the reference (64 ``tril``
    buffers, DDP broadcast_buffers=True) is gone — the masks are implicit;
  * gradients live in one flat fp32 buffer; each bucket is a contiguous slice
    (a whole transformer layer, the lm_head group, the embeddings) whose
    all-reduce is launched on a side stream as soon as the backward engine has
    enqueued that layer's last gradient kernel, so RCCL over xGMI overlaps the
    remaining backward. SUM all-reduce; the 1/world average is folded into the
    fused Adam kernel (grad_scale)."""
import torch
import torch.distributed as dist


class GradBuckets:
    def __init__(self, grads: torch.Tensor, ranges, group=None, on_reduced=None, force=False):
        """ranges: dict key -> (start, end) slices of ``grads``; keys are the
        notification ids passed to ``ready``. on_reduced(start, end, scale):
        called on the all-reduce side stream as soon as a bucket's SUM is in
        (the per-bucket optimizer: train_parallel.TrainStep runs the fused Adam
        over that slice there, so the last buckets' updates no longer queue
        behind one global Adam after the backward). force: issue the bucket
        collectives even at world size 1 (the RCCL path on one GPU: the SUM
        is then the identity, every stream dependency still runs)."""
        self.grads = grads
        self.ranges = dict(ranges)
        self.group = group
        self.on_reduced = on_reduced
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.force = force and dist.is_initialized()
        self.handles = []
        self.side = torch.cuda.Stream(device=grads.device) if grads.is_cuda else None

    def uncovered(self):
        """(start, end) slices of ``grads`` that no bucket covers"""
        out, pos = [], 0
        for s, e in sorted(self.ranges.values()):
            if s > pos:
                out.append((pos, s))
            pos = max(pos, e)
        if pos < self.grads.numel():
            out.append((pos, self.grads.numel()))
        return out

    def _reduce(self, buf, s, e):
        h = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        if self.on_reduced is None:
            self.handles.append(h)
            return
        h.wait()  # the current (side) stream waits for the collective, the host does not (RCCL)
        self.on_reduced(s, e, 1.0 / self.world)

    def ready(self, key):
        if (self.world == 1 and not self.force) or key not in self.ranges:
            return
        s, e = self.ranges[key]
        buf = self.grads[s:e]
        if self.side is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.grads.device))
            with torch.cuda.stream(self.side):
                self.side.wait_event(ev)
                self._reduce(buf, s, e)
        else:
            self._reduce(buf, s, e)

    def finish(self):
        """Blocks the current stream (not the host) until every bucket is
        reduced (and, with on_reduced, updated)."""
        for h in self.handles:
            h.wait()
        self.handles.clear()
        if self.side is not None:
            torch.cuda.current_stream(self.grads.device).wait_stream(self.side)
        return 1.0 / self.world

    def broadcast_params(self, flat: torch.Tensor, src=0):
        if self.world > 1 or self.force:
            dist.broadcast(flat, src=src, group=self.group)


def transformer_buckets(layout):
    """Bucket slices of the Transformer flat layout, keyed by the backward
    engine's hook ids: 'head' (ln_f + lm_head, ready first), layer ids L-1..0,
    and -1 (embeddings, ready last)."""
    from .transformer import _align
    import math
    off = layout.offsets
    n_layer = sum(1 for k in off if k.endswith(".ln1_w"))
    ranges = {}
    hs = off["lnf_w"][0]
    he = off["lm_b"][0] + _align(math.prod(off["lm_b"][1]))
    ranges["head"] = (hs, he)
    for l in range(n_layer):
        ranges[l] = layout.layer_range(l)
    ranges[-1] = (0, off["0.ln1_w"][0])
    return ranges
