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
from .config import LEARNING_RATE, Grammar
from .ddp import GradBuckets
from .loss import ce_forward_backward
from .transformer import Transformer, TransformerConfig


class TrainStep:
    """One optimisation step of train_parallel.py:173-183 (zero_grad, backward
    with DDP all-reduce, Adam(lr=5e-5)) for a Transformer or Mamba drop-in."""

    def __init__(self, model, lr=LEARNING_RATE, betas=(0.9, 0.999), eps=1e-8, grammar=None,
                 group=None):
        self.model = model
        self.eng = model.engine
        flat = model.flat.data
        self.grads = torch.zeros_like(flat)
        self.m = torch.zeros_like(flat)
        self.v = torch.zeros_like(flat)
        self.lr, self.betas, self.eps = lr, betas, eps
        self.grammar = grammar or Grammar()
        self.step_no = 0
        self.buckets = None
        if dist.is_initialized() and dist.get_world_size(group) > 1:
            self.buckets = GradBuckets(self.grads, self.eng.bucket_ranges(), group)
            self.buckets.broadcast_params(flat)
            self.eng.refresh_shadow(force=True)
            self.eng.layer_grad_ready = self.buckets.ready
        else:
            self.eng.layer_grad_ready = None

    def __call__(self, src, trg, meta):
        eng, cfg = self.eng, self.eng.cfg
        B, T = src.shape
        eng.forward(src, meta, train=self.model.training)
        A = eng.acts(B, T)
        dl = eng.dlogits_buffer(B, T)
        loss, _ = ce_forward_backward(src, A.logits.view(B, T, cfg.v_pad), trg, cfg.vocab_size, self.grammar,
                                      dlogits=dl.view(B, T, cfg.v_pad))
        self.grads.zero_()
        eng.backward(dl, self.grads)
        scale = self.buckets.finish() if self.buckets is not None else 1.0
        self.step_no += 1
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


def setup_distributed():
    """torchrun env -> (rank, local_rank, world); RCCL ("nccl") on MI355X."""
    if "RANK" in os.environ and not dist.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", 0))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
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


def train(model, type_name="transformer", data=None, steps=100, log_every=10, lr=LEARNING_RATE, save_dir=None,
          save_every=0):
    """Mirrors train_parallel.train: init RCCL, replicate the model, loop.
    data: an iterable of device batches (src, trg, meta) — e.g. the train
    loader of data.DatasetLoader — or None for synthetic grammar batches."""
    rank, local, world = setup_distributed()
    dev = torch.device("cuda", local)
    model.to(dev)
    step = TrainStep(model, lr=lr)
    if data is None:
        data = SyntheticMIDI(2, model.cfg.block_len, dev, rank)

    def batches():
        while True:  # epochs of a finite loader, as the reference's epoch loop
            n = 0
            for b in data:
                n += 1
                yield b
            if n == 0:
                raise ValueError("empty data loader")
    it = batches()
    t0 = time.time()
    log = []
    for i in range(steps):
        src, trg, meta = next(it)
        loss = step(src, trg, meta)
        if (i + 1) % log_every == 0 and rank == 0:
            log.append({"Step": i + 1, "Loss": f"{loss.item():.4f}", "elapsed_s": time.time() - t0})
            print(f"Step: {i + 1}, Loss: {log[-1]['Loss']}")
        if save_dir and save_every and (i + 1) % save_every == 0 and rank == 0:
            save_model(model, loss.item(), save_dir, type_name)
    return log
