"""Drop-in for train_parallel.py / train.py (the DDP training loop).

``train(model, type_name)`` keeps the reference's call shape and torchrun
environment (LOCAL_RANK / RANK / WORLD_SIZE, train_parallel.py:143-235) but
runs each iteration as ONE fused step on the MI355X engine:
  forward -> fused filtered-CE (loss + dlogits in one pass) -> backward with
  per-layer RCCL all-reduce buckets on a side stream -> fused Adam (+ bf16
  shadow refresh). No host sync per step (the reference calls loss.item()
  every step, train_parallel.py:185)."""
import os
import time

import numpy as np
import torch
import torch.distributed as dist

from . import ops
from .config import BLOCK_LEN, EPOCHS, EVAL_INTERVAL, LEARNING_RATE, SAVE_INTERVAL, Grammar
from .ddp import GradBuckets
from .loss import ce_forward_backward
from .transformer import Transformer, TransformerConfig


class TrainStep:
    """One optimisation step of train_parallel.py:173-183 (zero_grad, backward
    with DDP all-reduce, Adam(lr=5e-5)) for a Transformer or Mamba drop-in."""

    def __init__(self, model, lr=LEARNING_RATE, betas=(0.9, 0.999), eps=1e-8, grammar=None,
                 group=None, ddp=None):
        """ddp: None = bucketed all-reduce when the process group has more
        than one rank; True = also at world size 1 (the RCCL bucket path on
        one GPU; MSQ_DDP_BUCKETS=1 does the same)."""
        self.model = model
        self.eng = model.engine
        flat = model.flat.data
        self.grads = torch.zeros_like(flat)
        self.m = torch.zeros_like(flat)
        self.v = torch.zeros_like(flat)
        self.lr, self.betas, self.eps = lr, betas, eps
        self.grammar = grammar or Grammar()
        self.lm_bias_grad = self.eng.layout.views(self.grads)["lm_b"][:self.eng.cfg.vocab_size]
        self.step_no = 0
        if hasattr(self.eng, "head_stats"):  # the loss's column statistics from the lm_head epilogue
            self.eng.head_stats = True
        self.buckets = None
        # with world > 1 the fused Adam runs per bucket, on the all-reduce side
        # stream, as each bucket's SUM arrives (MSQ_GLOBAL_ADAM=1: one Adam over
        # the whole buffer after the backward); slices of an elementwise
        # update, so the parameters are bitwise those of the global step
        self.bucket_adam = os.environ.get("MSQ_GLOBAL_ADAM") != "1"
        if ddp is None:
            ddp = os.environ.get("MSQ_DDP_BUCKETS") == "1" or None
        if dist.is_initialized() and (ddp or dist.get_world_size(group) > 1):
            self.buckets = GradBuckets(self.grads, self.eng.bucket_ranges(), group,
                                       on_reduced=self._adam_slice if self.bucket_adam else None, force=bool(ddp))
            self.buckets.broadcast_params(flat)
            self.eng.refresh_shadow(force=True)
            self.eng.layer_grad_ready = self.buckets.ready
        else:
            self.eng.layer_grad_ready = None

    def _adam_slice(self, s, e, scale):
        sh = self.eng.shadow
        ops.adam_step(self.model.flat.data[s:e], self.grads[s:e], self.m[s:e], self.v[s:e], self.step_no, self.lr,
                      self.betas[0], self.betas[1], self.eps, shadow=sh[s:e] if sh is not None else None,
                      grad_scale=scale)

    def __call__(self, src, trg, meta):
        eng, cfg = self.eng, self.eng.cfg
        B, T = src.shape
        # the flat gradient is zero-filled on the Transformer forward's side
        # stream, under the forward
        eng.side_zero = [self.grads]
        try:
            eng.forward(src, meta, train=self.model.training)
        finally:
            eng.side_zero = None
        A = eng.acts(B, T)
        dl = eng.dlogits_buffer(B, T)
        if not getattr(eng, "side_zeroed", False):  # else zero-filled on the forward's side stream
            self.grads.zero_()
        # the output-bias gradient (column sums of dlogits) comes out of the loss pass
        loss, _ = ce_forward_backward(src, A.logits.view(B, T, cfg.v_pad), trg, cfg.vocab_size, self.grammar,
                                      dlogits=dl.view(B, T, cfg.v_pad), dbias=self.lm_bias_grad,
                                      colpart=A.colpart if getattr(A, "colpart_valid", False) else None)
        self.step_no += 1  # (the per-bucket Adam inside the backward uses it)
        eng.backward(dl, self.grads, head_bias_done=True)
        if self.buckets is not None and self.bucket_adam:
            scale = self.buckets.finish()
            for s, e in self.buckets.uncovered():
                self._adam_slice(s, e, scale)
        else:
            scale = self.buckets.finish() if self.buckets is not None else 1.0
            ops.adam_step(self.model.flat.data, self.grads, self.m, self.v, self.step_no, self.lr, self.betas[0],
                          self.betas[1], self.eps, shadow=eng.shadow, grad_scale=scale)
        eng.mark_shadow_fresh()
        return loss


class SyntheticMIDI:
    """Grammar-cycled synthetic token batches, generated on
    the host once and kept resident in HBM; seed 1234 + rank."""

    COMPOSERS = [[519, 279, 202, 202, 202, 178], [432, 277, 202, 202, 202, 173], [437, 279, 272, 202, 202, 180],
                 [452, 272, 202, 202, 202, 184], [508, 272, 202, 202, 202, 184]]

    def __init__(self, B, T, device, rank=0, n_batches=4, grammar: Grammar = None):
        grammar = grammar or Grammar()
        s = grammar.disc.start_idx
        V = grammar.disc.vocab_size
        rng = np.random.default_rng(1234 + rank)
        self.batches = []
        for n in range(n_batches):
            L = B * (T + 1) + 8
            toks = []
            while len(toks) < L:
                toks += [rng.integers(s["pitch"], s["dyn"]), rng.integers(s["dyn"], s["length"]),
                         rng.integers(s["length"], s["time"])]
                if rng.random() < 0.5:
                    toks.append(rng.integers(s["time"], s["tempo"]))
                toks.append(rng.integers(s["tempo"], V))
            w = torch.tensor(np.asarray(toks[:B * (T + 1)], dtype=np.int64)).view(B, T + 1)
            meta = torch.tensor([self.COMPOSERS[(n * B + b) % 5] for b in range(B)], dtype=torch.int64)
            self.batches.append((w[:, :-1].contiguous().to(device), w[:, 1:].contiguous().to(device), meta.to(device)))

    def __iter__(self):
        while True:
            for b in self.batches:
                yield b


def setup_distributed(backend=None):
    """torchrun env (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*) -> (rank,
    local_rank, world). backend "nccl" (= RCCL over xGMI on MI355X, the
    default) binds the process to GPU LOCAL_RANK first (train_parallel.py:
    144-145); "gloo" touches no GPU (CPU tests and dry runs)."""
    if "RANK" in os.environ and not dist.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", 0))
        backend = backend or "nccl"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    if dist.is_initialized():
        return dist.get_rank(), int(os.environ.get("LOCAL_RANK", 0)), dist.get_world_size()
    return 0, 0, 1


def new_model(type_name="transformer", precision="bf16", **kw):
    """train_parallel.py:56-65: "transformer" | "mamba" (xlstm is out of scope)."""
    if type_name == "mamba":
        from .mamba import Mamba
        return Mamba(precision=precision, **kw)
    if type_name != "transformer":
        raise NotImplementedError(f"model type {type_name!r} is not on the MI355X path (see DESIGN.md)")
    return Transformer(TransformerConfig(precision=precision, **kw))


def save_model(model, loss, pretrained_path, type_name="transformer"):
    """train.py:69-77: state_dict (the reference's keys, incl. the tril
    buffers) to <pretrained>/<type>/loss_<loss>_time_<now>.pth."""
    from datetime import datetime
    now = datetime.now().strftime("%Y-%m-%d-%H-%M-%S")
    path = os.path.join(pretrained_path, type_name, f"loss_{loss:.2f}_time_{now}.pth")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    torch.save({k: v.detach().cpu() for k, v in model.state_dict().items()}, path)
    return path


def load_model(type_name, path, precision="bf16", device="cuda", **kw):
    """train.py:63-67 (load_model): a reference-format .pth (per-head
    key/query/value, tril buffers) into the MI355X engine. Loaded with
    weights_only=True: nothing in the file is executed."""
    model = new_model(type_name, precision=precision, **kw)
    model.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
    return model.to(device)


def evaluate(model, loader, grammar=None):
    """The validation pass of train_parallel.py:197-207: model.eval(), forward
    + filtered CE under no_grad over the test loader, averaged over its
    batches (a device scalar; the caller decides when to sync)."""
    from .loss import filtered_cross_entropy
    was = model.training
    model.eval()
    total, n = None, 0
    with torch.no_grad():
        for src, trg, meta in loader:
            l = filtered_cross_entropy(src, model(src, meta), trg, grammar)
            total = l if total is None else total + l
            n += 1
    model.train(was)
    if n == 0:
        return None
    return total / n


def _epoch_batches(data, steps_per_epoch):
    """One epoch of ``data``: a finite loader (len() batches, the reference's
    DataLoader) or ``steps_per_epoch`` batches of an endless stream."""
    if hasattr(data, "__len__") and not isinstance(data, SyntheticMIDI):
        yield from data
        return
    it = iter(data)
    for _ in range(steps_per_epoch):
        yield next(it)


def train(model, type_name="transformer", data=None, test_data=None, epochs=EPOCHS, max_steps=None,
          eval_interval=EVAL_INTERVAL, save_interval=SAVE_INTERVAL, lr=LEARNING_RATE, save_dir=None, log_file=None,
          steps_per_epoch=100, grammar=None):
    """Mirrors train_parallel.train (train_parallel.py:143-235): init RCCL,
    replicate the model (one parameter broadcast), then per epoch: model.train()
    and a pass over the train loader (loss logged every ``eval_interval`` steps
    on rank 0), the epoch's average loss, model.eval() + validation loss under
    no_grad over ``test_data``, a rank-0 save every ``save_interval`` epochs
    named by the average validation loss, and on exit (normal end, max_steps,
    or KeyboardInterrupt) a final rank-0 save and log dump.

    data / test_data: iterables of device batches (src, trg, meta) — e.g.
    ``data.DatasetLoader(...).get_dataloaders()`` — or None for synthetic
    grammar batches (``steps_per_epoch`` of them per epoch). The per-step loss
    stays on the device; the host reads it only at the log points (the
    reference syncs with loss.item() every step, :185)."""
    from datetime import datetime
    import json
    rank, local, world = setup_distributed()
    dev = torch.device("cuda", local)
    model.to(dev)
    step = TrainStep(model, lr=lr, grammar=grammar)
    if data is None:
        data = SyntheticMIDI(2, getattr(model.cfg, "block_len", BLOCK_LEN), dev, rank)
    log = []

    def note(msg):
        if rank == 0:
            print(msg)
            log.append({"timestamp": str(datetime.now()), "message": msg})

    def dump():
        if rank == 0 and log_file:
            os.makedirs(os.path.dirname(os.path.abspath(log_file)), exist_ok=True)
            with open(log_file, "w") as f:
                json.dump(log, f, indent=2)

    note("Training started!")
    avg_val = None
    n_steps = 0
    done = False
    try:
        for epoch in range(epochs):
            model.train()
            total, nb = None, 0
            for src, trg, meta in _epoch_batches(data, steps_per_epoch):
                loss = step(src, trg, meta)
                total = loss.detach().clone() if total is None else total + loss.detach()
                nb += 1
                n_steps += 1
                if nb % eval_interval == 0 and rank == 0:
                    msg = f"{loss.item():.4f}"
                    log.append({"Step": n_steps, "Loss": msg})
                    print(f"Step: {n_steps}, Loss: {msg}")
                if max_steps is not None and n_steps >= max_steps:
                    done = True
                    break
            if nb == 0:
                raise ValueError("empty data loader")
            note(f"Epoch [{epoch + 1}/{epochs}], Average Loss: {(total / nb).item():.4f}")
            if test_data is not None:
                v = evaluate(model, test_data, grammar)
                if v is not None:
                    avg_val = v.item()
                    note(f"Epoch [{epoch + 1}/{epochs}], Validation Loss: {avg_val:.4f}")
            if save_dir and (epoch + 1) % save_interval == 0 and rank == 0:
                save_model(model, avg_val if avg_val is not None else 0.0, save_dir, type_name)
                dump()
            if done:
                break
    except KeyboardInterrupt:
        if rank == 0:
            print("Interrupted!")
    finally:
        if rank == 0 and save_dir:
            print("Saving model before exit...")
            save_model(model, avg_val if avg_val is not None else 0.0, save_dir, type_name)
        note("Training complete!")
        dump()
    return log
