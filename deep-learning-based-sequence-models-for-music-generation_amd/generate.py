"""Drop-in for scripts/generate.py:14-95 (``generate``) on the MI355X engine.

Exact sliding-window mode (the reference's semantics): every step runs the
full forward over the last ``context_len`` tokens (the Transformer is
length-anchored: its relative positions are measured from the window end, so
a KV cache cannot reproduce this loop), takes the filtered
logit of the last row (its log-softmax runs over the whole window's time
axis), applies the repetition penalties, picks k with Python's ``random``
exactly like the reference (same call order, so seeded runs draw the same
k's) and samples on the device by inverse CDF on a uniform per row (replacing
torch.multinomial). The history stays on the device; the only per-step
device->host traffic is the B last tokens needed for the host-side k choice.

Cached mode (``mode="cached"``):
* Mamba: while the window still holds the whole
  history (prompt + generated <= context_len) every Mamba2 mixer is causal and
  the final LayerNorm / head are per position, so the logits of the new last
  row equal one recurrent step from the mixer states after the previous row,
  and the time-axis log-softmax of filtered_logit only needs a running
  per-vocabulary LSE. The prompt is prefilled by one full forward (which also
  leaves the states); each later step is one ``MambaEngine.step``. EXACT; once
  the window starts to slide the loop falls back to the exact full forward.
* Transformer (BASELINE cfg 5 "KV-cache AR decode"): a documented
  APPROXIMATION (the model is length-anchored). The prompt
  window is prefilled exactly (its first sampled token equals the exact
  mode's); every later token is computed once, as the last row of its own
  window (skew term q . R[j], j = the key's window position), against the
  cached keys / values of the window, which then slides over a ring of
  ``context_len`` tokens; filtered_logit's time-axis LSE runs over the
  window's cached logits rows. oracle/transformer.py CachedTransformer
  restates these semantics; tests/test_decode_cached_gpu.py pins the build to it.

Sharded decode (``group=``): the global batch of world x B
prompts is split by rows over the ranks of a process group, one model
replica per GPU. The only exchange is the host-side k choice: the reference
draws ``random.choice`` for every row in row order each step, so every rank
all-gathers the world x B last tokens (one small collective per step) and
replays that whole sequence, then keeps its own rows' k's; the per-row
uniforms are drawn for all world x B rows from the same seed and sliced the
same way. Rank r's rows are then bit for bit rows r*B .. r*B+B-1 of a single
process run over the concatenated batch with the same seeds
(tests/test_decode_shard_gpu.py).
"""
import random as _random

import torch
import torch.distributed as dist

from . import _lib as L
from ._lib import ptr, call, stream, dt
from .config import Grammar
from .loss import grammar_table
from .ops import workspace


def choose_k(last_tokens, start, rng):
    """generate.py:47-56 — consumes ``rng`` only for tempo/dyn/pitch tokens."""
    ks = []
    for t in last_tokens:
        if t >= start["tempo"]:
            ks.append(rng.choice([1, 1, 1, 2, 2]))
        elif t >= start["time"] or t >= start["length"]:
            ks.append(1)
        elif t >= start["dyn"]:
            ks.append(rng.choice([1, 3]))
        else:
            ks.append(rng.choice([1, 2]))
    return ks


class _Shard:
    """Row shard of a decode over a process group (module docstring)."""

    def __init__(self, group, B, dev):
        if not dist.is_initialized():
            raise RuntimeError("generate(group=...) needs an initialised torch.distributed process group")
        if group is True:
            group = None  # the default group
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.gloo = dist.get_backend(group) == "gloo"
        self.dev = dev
        sizes = self.gather(torch.tensor([B], dtype=torch.int64, device=dev))
        if any(n != B for n in sizes):
            raise ValueError(f"sharded generate needs the same batch on every rank, got {sizes}")
        self.B = B
        self.lo, self.hi = self.rank * B, (self.rank + 1) * B

    def gather(self, t):
        """all-gather of a small int64 device vector -> host list, rank order"""
        t = t.cpu() if self.gloo else t.contiguous()
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t, group=self.group)
        return torch.cat(parts).tolist()


@torch.no_grad()
def generate(model, context_len, token_ids, meta_ids, num_tokens=1000, device="cuda", rng=None, uniforms=None,
             grammar: Grammar = None, return_tensor=False, mode="exact", group=None):
    """Returns a list of B token lists of length T0 + num_tokens (like the
    reference). ``rng`` defaults to the global ``random`` module (as in the
    reference); ``uniforms`` is an optional iterator of floats (one per row
    per step, rows in order) for reproducible sampling, else a device
    torch.Generator is used. ``group`` (a torch.distributed process group, or
    True for the default one): this call decodes this rank's B rows of a
    sharded batch of world x B rows (module docstring); ``rng``, ``uniforms``
    (world x B per step) and torch's seed must then be the same on every rank."""
    grammar = grammar or Grammar()
    rng = rng or _random
    eng = model.engine
    cfg = eng.cfg
    V = cfg.vocab_size
    start = grammar.disc.start_idx
    dev = torch.device(device)
    token_ids = token_ids.to(dev)
    meta_ids = meta_ids.to(dev).contiguous()
    B, T0 = token_ids.shape
    ldh = T0 + num_tokens + 1
    hist = torch.zeros(B, ldh, dtype=torch.int64, device=dev)
    hist[:, :T0] = token_ids
    out_tok = torch.empty(B, dtype=torch.int64, device=dev)
    wtab = grammar_table(dev, grammar)
    b = grammar.bounds
    shard = _Shard(group, B, dev) if group is not None else None
    nrow = shard.world * B if shard else B  # rows the host-side RNG replays per step
    last_host = shard.gather(token_ids[:, -1]) if shard else token_ids[:, -1].tolist()
    gen = None
    if mode not in ("exact", "cached"):
        raise ValueError(f"mode must be 'exact' or 'cached', not {mode!r}")
    cached = mode == "cached"
    slides = cached and getattr(eng, "cache_slides", False)  # Transformer: stays cached past the context
    cache = None
    ldz = (V + 3) // 4 * 4
    z = torch.empty(B, 1, ldz, device=dev, dtype=torch.float32)
    # host <-> device staging of the per-step host work (pinned: the copies
    # stay asynchronous and ordered on their streams)
    kt_host = torch.empty(B, dtype=torch.int32, pin_memory=True)
    kt = torch.empty(B, dtype=torch.int32, device=dev)
    u_host = torch.empty(nrow, dtype=torch.float32, pin_memory=True)
    u_dev = torch.empty(nrow, dtype=torch.float32, device=dev)
    # Cached steps are pipelined (unsharded): the sampled tokens of step s go
    # to the host on a side stream while step s+1's recurrent / cached forward
    # (which reads them on the device) already runs, so the host-side k choice
    # (Python's random, as in the reference) overlaps the device work instead
    # of following it
    pipelined = shard is None
    tok_host = torch.empty(B, dtype=torch.int64, pin_memory=True)
    side = torch.cuda.Stream(device=dev) if pipelined else None
    prefetched = False

    def cached_at(c):
        return cached and cache is not None and (c <= context_len or slides)

    def launch_step():
        # one recurrent position: the token sampled last step (out_tok) at row cur-1
        lg = eng.step(out_tok, cache)
        call("msq_filtered_logit_step", ptr(z), ldz, ptr(cache.lse), ptr(lg), dt(lg), lg.stride(0),
             ptr(out_tok), ptr(wtab), b[0], b[1], b[2], b[3], B, V, stream())

    for step in range(num_tokens):
        cur = T0 + step
        W = min(cur, context_len)
        if cached_at(cur):
            if not prefetched:
                launch_step()
        else:
            window = hist[:, cur - W:cur].contiguous()
            if cached and cache is None and (cur <= context_len or slides):  # prefill, states left in the cache
                cache = eng.decode_cache(B, context_len) if slides else eng.decode_cache(B)
                logits = eng.forward(window, meta_ids, save=False, cache=cache)
                col_lse = cache.lse
            else:
                logits = eng.forward(window, meta_ids, save=False)
                col_lse = torch.empty(B, V, device=dev, dtype=torch.float32)
            A = eng.acts(B, W, save=False)
            ws = workspace(L.lib().msq_filtered_workspace(B, W, V), dev, "loss")
            call("msq_filtered_logit", ptr(z), ldz, ptr(A.logits), dt(A.logits), cfg.v_pad, ptr(window), ptr(wtab),
                 b[0], b[1], b[2], b[3], B, W, V, W - 1, ptr(col_lse), ptr(ws), stream())
            del logits
        prefetched = False
        ks = choose_k(last_host, start, rng)
        if uniforms is not None:
            u_host.numpy()[:] = [next(uniforms) for _ in range(nrow)]
            u_dev.copy_(u_host, non_blocking=True)
            u = u_dev
        else:
            if gen is None:
                # the reference samples with torch.multinomial, i.e. from torch's
                # global RNG, and draws only the k's from Python's random: seed
                # the device stream from torch's CPU generator so ``rng`` sees
                # exactly the reference's random.choice sequence
                gen = torch.Generator(device=dev)
                gen.manual_seed(int(torch.randint(0, 2 ** 62, (1,)).item()))
            u = torch.rand(nrow, device=dev, generator=gen)
        if shard:
            ks, u = ks[shard.lo:shard.hi], u[shard.lo:shard.hi].contiguous()
        kt_host.numpy()[:] = ks
        kt.copy_(kt_host, non_blocking=True)
        call("msq_decode_sample", ptr(hist), ldh, cur, ptr(z), ldz, B, V, ptr(kt), ptr(u), ptr(out_tok),
             start["dyn"], start["length"], start["time"], start["tempo"], stream())
        # the one device->host transfer per step (host-side k choice); sharded: all ranks' rows
        if shard:
            last_host = shard.gather(out_tok)
            continue
        main = torch.cuda.current_stream(dev)
        sampled = torch.cuda.Event()
        sampled.record(main)
        side.wait_event(sampled)
        with torch.cuda.stream(side):
            tok_host.copy_(out_tok, non_blocking=True)
            landed = torch.cuda.Event()
            landed.record(side)
        if step + 1 < num_tokens and cached_at(cur + 1):
            launch_step()
            prefetched = True
        landed.synchronize()
        last_host = tok_host.tolist()
    seq = hist[:, :T0 + num_tokens]
    return seq if return_tensor else seq.tolist()
