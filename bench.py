"""Headline benchmark: MIDI tokens/s of the Transformer training step
(configs/transformer default: d=1024, 8 heads, 8 layers, T=2048 (+6 meta),
V=17914) at B=32 per GPU, bf16 MFMA path, synthetic grammar-cycled tokens,
random-init weights. One process per GPU (torchrun); weak scaling.

Prints ONE JSON line on rank 0 (contract in the task statement)."""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def launch_ranks():
    """`python bench.py --gpus N` (N > 1) without a torchrun environment:
    start N worker ranks as ONE child process (torch.distributed.run, one
    process per GPU, rendezvous on 127.0.0.1), relay their output and exit
    with their status. Runs before this process imports torch, so the parent
    never touches a GPU (and never execs)."""
    if "RANK" in os.environ:
        return
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    n = ap.parse_known_args()[0].gpus
    if n <= 1:
        return
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


if __name__ == "__main__":
    launch_ranks()

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import _pkgload  # noqa: E402

_pkgload.load()
from midiseq import ops  # noqa: E402
from midiseq import _lib as L  # noqa: E402
from midiseq.transformer import Transformer, TransformerConfig  # noqa: E402
from midiseq.train_parallel import TrainStep, SyntheticMIDI, setup_distributed  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
METRIC = "MIDI tokens/sec/GPU (train, seq_len=2048) + AR decode tokens/sec at 1/2/4/8 GPU"
def flops_per_token(cfg, T):
    """Algorithmic training FLOPs per MIDI token (SURVEY.md §8(d) cfg 2):
    3 x forward; forward = L (24 S d^2 + 3 d S (S+1)) + 2 T d V per sequence."""
    S, d = T + 6, cfg.n_embd
    fwd = cfg.n_layer * (24 * S * d * d + 3 * d * S * (S + 1)) + 2 * T * d * cfg.vocab_size
    return 3.0 * fwd / T


def _gemm_class(a):
    """msq_gemm / msq_gemm_ex / msq_gemm_dropout args -> (class, FLOPs); the
    dX products are labelled by their caller (ops.gemm(role="gemm_dX"))."""
    ta, tb, M, N, K, batch, epi = a[1], a[2], a[3], a[4], a[5], a[16], a[17]
    cls = "gemm_dW" if epi == L.EPI_ACCUM else (L.ROLE or ("gemm_dX" if (tb and not ta) else "gemm_fwd"))
    return cls, 2.0 * M * N * K * batch, None


def _attn_flops(B, S, H, hs):
    """QK^T, q.R^T and PV over the causal triangle (SURVEY.md §8(d) cfg 2)."""
    return 3 * 2.0 * hs * S * (S + 1) / 2 * B * H


CLASSIFY = {
    "msq_gemm": _gemm_class, "msq_gemm_ex": _gemm_class, "msq_gemm_dropout": _gemm_class,
    "msq_relattn_fwd_dropout": lambda a: ("attn_fwd", _attn_flops(a[7], a[8], a[9], a[10]), None),
    # backward = 2 x the forward's products (algorithmic; the recompute of P is not counted)
    "msq_relattn_bwd_dropout": lambda a: ("attn_bwd", 2 * _attn_flops(a[11], a[12], a[13], a[14]), None),
    "msq_relattn_bwd_ws": lambda a: ("attn_bwd", 2 * _attn_flops(a[11], a[12], a[13], a[14]), None),
    # FFN dX with the FFN1 bias gradient in its epilogue
    "msq_gemm_colsum": lambda a: ("gemm_dX", 2.0 * a[2] * a[3] * a[4], None),
    # filtered CE: 3 reads of the logits + 1 write of dlogits ([B, T, ld] of the act dtype)
    "msq_filtered_ce": lambda a: ("loss", None, 4.0 * a[13] * a[14] * a[5] * (2 if a[4] == L.BF16 else 4)),
    "msq_filtered_ce_bias": lambda a: ("loss", None, 4.0 * a[14] * a[15] * a[6] * (2 if a[5] == L.BF16 else 4)),
    # the same with the column statistics from the lm_head epilogue: 2 reads of the logits + 1 write
    "msq_filtered_ce_bias_part": lambda a: ("loss", None, 3.0 * a[14] * a[15] * a[6] * (2 if a[5] == L.BF16 else 4)),
    # lm_head forward with the column (max, sum exp) partials in its epilogue
    "msq_gemm_bias_colstats": lambda a: ("gemm_fwd", 2.0 * a[1] * a[2] * a[3], None),
    "msq_layernorm_fwd": lambda a: ("layernorm", None, None),
    "msq_layernorm_bwd": lambda a: ("layernorm", None, None),
    "msq_layernorm_bwd_dropout": lambda a: ("layernorm", None, None),
    "msq_colsum": lambda a: ("colsum", None, None),
    # 4 fp32 reads (p, g, m, v) + 3 fp32 writes + 1 bf16 shadow write per parameter
    "msq_adam_step": lambda a: ("adam", None, 30.0 * a[5]),
    "msq_dropout_attn_mask": lambda a: ("dropout_mask", None, None),
    "msq_embed_fwd": lambda a: ("embed", None, None), "msq_embed_bwd": lambda a: ("embed", None, None),
    # SSD scan (SURVEY.md §8(d) cfg 3): bf16 x, B, C, dt in + y out = 8 512 B per token per layer (d_inner 2048)
    "msq_mamba_ssd_fwd_state": lambda a: ("ssd_fwd", None, (4 * a[14] + 4 * 64 + 2 * a[15]) * float(a[12] * a[13])),
    # the rest of the Mamba2 mixer, bytes per token per layer as the kernels move
    # them (Mamba byte model; N = 64 states, conv_dim = di + 128):
    # ssd_bwd: dy bf16 (the compute dtype, since 840be59) + xc bf16 + dt + chunk
    #          states f32 (H P N 4 / 64 tokens) in, dxc f32 + ddt out
    "msq_mamba_ssd_bwd": lambda a: ("ssd_bwd", None, float(a[17] * a[18]) * (
        2 * a[19] + 2 * (a[19] + 128) + 2 * a[20] + a[20] * 64 * 64 * 4 / 64 + 4 * (a[19] + 128) + 2 * a[20])),
    # conv fwd: xBC bf16 in, xc bf16 out; bwd: dxc f32 + xBC bf16 in, dxBC bf16 out
    "msq_mamba_conv_fwd": lambda a: ("mamba_conv", None, float(a[7] * a[8]) * 4 * (a[9] + 128)),
    "msq_mamba_conv_bwd": lambda a: ("mamba_conv", None, float(a[10] * a[11]) * 8 * (a[12] + 128)),
    # gated RMSNorm fwd: y bf16 + z bf16 in, yn bf16 + rstd out; bwd: y bf16, z, dyn f32 in, dy f32, dz out
    "msq_mamba_gnorm_fwd": lambda a: ("mamba_gnorm", None, float(a[9]) * (2 * a[10] + 2 * a[10] + 2 * a[10] + 4)),
    "msq_mamba_gnorm_bwd": lambda a: ("mamba_gnorm", None, float(a[12]) * (2 + 2 + 4 + 4 + 2) * a[13]),
}


PMC_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r6")


def pmc_traffic(cls, name="pmc_traffic.json"):
    """HBM bytes per launch of a kernel class from the committed PMC passes
    (tools/pmc_traffic.py, profiles/r6/<name>), or None."""
    try:
        with open(os.path.join(PMC_DIR, name)) as f:
            c = json.load(f)["classes"].get(cls)
        return round(c["hbm_bytes_per_launch"]) if c else None
    except (OSError, ValueError, KeyError):
        return None


class ClassTimer:
    """HIP events around every libmidiseq launch (midiseq._lib.TAP), recorded
    on the stream the launch goes to (torch's current stream at the call:
    the main stream, or the weight-gradient / side stream inside its
    `with torch.cuda.stream(...)` block), grouped by kernel class."""

    def __init__(self):
        self.rec, self.on = [], False

    def __call__(self, name, args, launch):
        if not self.on:
            return launch()
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        r = launch()
        e.record()
        cls, flops, nbytes = CLASSIFY.get(name, lambda a: ("other:" + name[4:], None, None))(args)
        self.rec.append((cls, flops, nbytes, s, e))
        return r

    def table(self, steps):
        """{class: {launches_per_step, ms_per_step, avg_launch_ms, achieved, peak, unit, frac}}."""
        agg = {}
        for cls, flops, nbytes, s, e in self.rec:
            a = agg.setdefault(cls, {"n": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0, "f": flops is not None,
                                     "b": nbytes is not None})
            a["n"] += 1
            a["ms"] += s.elapsed_time(e)
            a["flops"] += flops or 0.0
            a["bytes"] += nbytes or 0.0
        out = {}
        for cls, a in sorted(agg.items(), key=lambda kv: -kv[1]["ms"]):
            row = {"launches_per_step": round(a["n"] / steps, 2), "ms_per_step": round(a["ms"] / steps, 3),
                   "avg_launch_ms": round(a["ms"] / a["n"], 4)}
            if a["f"]:
                ach = a["flops"] / (a["ms"] * 1e-3) / 1e12
                row.update(bound="mfma", achieved=round(ach, 1), peak=PEAK_BF16_TFLOPS, unit="TFLOP/s",
                           frac=round(ach / PEAK_BF16_TFLOPS, 4), work_per_launch=a["flops"] / a["n"])
            elif a["b"]:
                ach = a["bytes"] / (a["ms"] * 1e-3) / 1e9
                row.update(bound="hbm", achieved=round(ach, 1), peak=PEAK_HBM_GBS, unit="GB/s",
                           frac=round(ach / PEAK_HBM_GBS, 4), work_per_launch=a["bytes"] / a["n"])
            out[cls] = row
        return out


CALIB = os.path.join(ROOT, "profiles", "r2", "cpu_calibration.json")


def _oracle_train_rate(hp, B, T, budget_s, max_steps):
    """tokens/s of the oracle's fp32 train step (forward, filtered CE,
    backward, Adam) on this host; one untimed warm-up step."""
    import numpy as np
    from oracle import loss as oloss, transformer as otr
    from oracle.fill import REAL, grammar_tokens
    shapes = otr.param_shapes(hp["n_embd"], hp["n_heads"], hp["n_layer"], hp["block_len"], REAL.size, 568)
    g = torch.Generator().manual_seed(0)
    p = {k: (torch.randn(s, generator=g) * 0.02).requires_grad_(True) for k, s in shapes.items()}
    opt = torch.optim.Adam(list(p.values()), lr=5e-5)
    rng = np.random.default_rng(0)
    w = np.stack([grammar_tokens(rng, REAL, T + 1) for _ in range(B)])
    src, trg = torch.from_numpy(w[:, :-1].copy()), torch.from_numpy(w[:, 1:].copy())
    meta = torch.tensor([[519, 279, 202, 202, 202, 178]] * B)

    def step():
        loss = oloss.loss(src, trg, otr.forward(p, src, meta, hp["n_layer"], hp["n_heads"]), REAL)
        opt.zero_grad()
        loss.backward()
        opt.step()
    step()
    steps, t0 = 0, time.time()
    while True:
        step()
        steps += 1
        if time.time() - t0 > budget_s or steps >= max_steps:
            break
    return steps * B * T / (time.time() - t0), steps


def cpu_baseline():
    """The CPU oracle (plain PyTorch fp32 restatement of the reference's train
    step, the 'port') timed on this host's cores: cfg 2's model at B=1
    (headline) and cfg 1 (2 layers, d 128, T 256, B 2). The restatement-to-
    reference ratio measured in the build container on the same cores for both
    (tools/calibrate_cpu.py -> profiles/r2/cpu_calibration.json) gives the
    reference-equivalent rate beside it."""
    nproc = os.cpu_count() or 1
    # at most 16 threads: the GPU box gives a job a 16-CPU share of a larger
    # host (os.cpu_count() reports the whole machine)
    threads = min(16, nproc)
    torch.set_num_threads(threads)
    v2, n2 = _oracle_train_rate(dict(n_embd=1024, n_heads=8, n_layer=8, block_len=2048), 1, 2048, 15.0, 3)
    v1, n1 = _oracle_train_rate(dict(n_embd=128, n_heads=8, n_layer=2, block_len=256), 2, 256, 5.0, 30)
    out = {"value": round(v2, 2), "unit": "MIDI tokens/s", "cores": threads, "host_cpus": nproc, "kind": "port",
           "sample": f"oracle/ fp32 train step (fwd+filtered CE+bwd+Adam), default model, B=1, T=2048, {n2} steps",
           "cfg1": {"value": round(v1, 1), "unit": "MIDI tokens/s",
                    "sample": f"oracle/ fp32 train step, 2 layers d=128 h=8, B=2, T=256, {n1} steps"}}
    try:
        with open(CALIB) as f:
            cal = json.load(f)
        r1, r2 = cal["configs"]["cfg1"], cal["configs"]["cfg2_b1"]
        out["calibration"] = {
            "source": "profiles/r2/cpu_calibration.json (build container, same cores for both)",
            "threads": cal["threads"], "oracle_over_reference_cfg1": r1["oracle_over_reference"],
            "oracle_over_reference_cfg2": r2["oracle_over_reference"],
            "reference_s_per_step_cfg1": r1["reference_s_per_step"], "reference_s_per_step_cfg2": r2["reference_s_per_step"],
            "reference_equiv_value": round(v2 * r2["oracle_over_reference"], 2),
            "reference_equiv_cfg1": round(v1 * r1["oracle_over_reference"], 1)}
    except (OSError, KeyError, ValueError):
        pass
    return out


def timed(fn, steps, warmup, world, dev):
    """Runs fn() warmup times untimed, then steps times between barrier +
    synchronize brackets; returns the max-over-ranks wall seconds."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    return el


def _group(world):
    """decode legs: rows sharded over the default group (generate(group=True))"""
    return True if world > 1 else None


def _fwd_flops(cfg, T):
    """algorithmic forward FLOPs of one sequence (SURVEY.md §8(d) cfg 2)"""
    S, d = T + 6, cfg.n_embd
    return cfg.n_layer * (24 * S * d * d + 3 * d * S * (S + 1)) + 2 * T * d * cfg.vocab_size


def decode_leg(dev, rank, world, steps=3, B=64, T=2048):
    """Config 5: B=64 composer-conditioned prompts of 2048 tokens per GPU
    (the global batch of world x 64 rows sharded by row: generate(group=...),
    one all-gather of the last tokens per step for the host-side k choice),
    exact sliding-window decode (full forward + filtered logit + penalties +
    top-k + sampling per new token)."""
    import random
    from midiseq.generate import generate
    m = Transformer(TransformerConfig(precision="bf16", dropout=0.0)).to(dev)
    src, _, meta = SyntheticMIDI(B, T, dev, rank, n_batches=1).batches[0]
    el = timed(lambda: generate(m, T, src, meta, num_tokens=1, rng=random.Random(0), device=dev,
                                group=_group(world)), steps, 1, world, dev)
    flops = B * _fwd_flops(m.cfg, T)  # SURVEY.md §8(d) cfg 5: 64 x F_fwd = 37.9 TFLOP per step
    del m
    ach = flops / (el / steps) / 1e12
    return {"value": round(world * B * steps / el, 2), "unit": "new tokens/s", "ms_per_token_step": round(el / steps * 1e3, 3),
            "roofline": {"kernel": "whole decode step (full forward of the window + filtered logit + sampler)",
                         "bound": "mfma", "achieved": round(ach, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(ach / PEAK_BF16_TFLOPS, 4), "traffic": None,
                         "algorithmic_work_per_step": flops},
            "config": {"workload": "cfg 5 exact sliding-window decode (full fwd per step)", "batch_per_gpu": B,
                       "context": T}}


def mamba_decode_leg(dev, rank, world, B=64, T0=1024, K=64, steps=2):
    """Mamba (d=1024, 10 layers, bf16) cached decode of
    B=64 prompts of T0 tokens per GPU (replicas): one prefill forward, then
    one recurrent step per new token. Steady-state rate = K new tokens per
    row over (time of prefill + K steps) - (time of prefill alone)."""
    import random
    from midiseq.generate import generate
    from midiseq.mamba import Mamba
    m = Mamba(precision="bf16").to(dev)
    src, _, meta = SyntheticMIDI(B, T0, dev, rank, n_batches=1).batches[0]
    run = lambda n: generate(m, 2048, src, meta, num_tokens=n, rng=random.Random(0), device=dev,  # noqa: E731
                             mode="cached", group=_group(world))
    el_pre = timed(lambda: run(1), steps, 1, world, dev)
    el_all = timed(lambda: run(1 + K), steps, 1, world, dev)
    el_exact = timed(lambda: generate(m, 2048, src, meta, num_tokens=1, rng=random.Random(0), device=dev,
                                      group=_group(world)), steps, 1, world, dev)
    del m
    ms_step = (el_all - el_pre) / (steps * K) * 1e3
    return {"value": round(world * B / (ms_step * 1e-3), 1), "unit": "new tokens/s", "ms_per_token_step": round(ms_step, 3),
            "prefill_ms": round(el_pre / steps * 1e3, 2), "exact_full_forward_ms_per_step": round(el_exact / steps * 1e3, 2),
            "config": {"workload": "Mamba cached decode (recurrent step, exact while prompt+new <= context)",
                       "batch_per_gpu": B, "prompt": T0, "new_tokens": K, "context": 2048}}


def midi_decode_leg(dev, rank, world, B=64, L=4048, iters=50, cpu_rows=4):
    """token -> note decode (processing.decode +
    revert_note_time) of the B=64 generated rows of cfg 5 (2048 prompt + 2000
    new tokens, generate_midi_combined --retain) while they are in HBM: one
    msq_midi_decode launch per batch, timed with HIP events on its stream.
    Algorithmic bytes: 8 B read per token + 48 B written per note.
    cpu_baseline: the oracle's per-row Python decode (the reference's loop) on
    cpu_rows rows, scaled to tokens/s."""
    from midiseq import midi
    rows = SyntheticMIDI(B, L, dev, rank, n_batches=1).batches[0][0].contiguous()
    nb = midi.decode_batch(rows)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        midi.decode_batch(rows, out=nb)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    notes = int(nb.count.sum())
    nbytes = B * L * 8 + notes * 48
    out = {"value": round(world * B * L / (ms * 1e-3), 1), "unit": "tokens/s", "ms_per_batch": round(ms, 4),
           "notes_per_batch": notes, "achieved_GBps": round(nbytes / (ms * 1e-3) / 1e9, 1), "peak_GBps": 8000.0,
           "config": {"workload": "token->note decode of cfg 5 generated rows (msq_midi_decode)", "batch_per_gpu": B,
                      "row_tokens": L}}
    if rank == 0:
        from oracle import midi as omidi
        from midiseq.config import DEFAULT_DISC
        rows_np = rows[:cpu_rows].cpu().numpy()
        t0 = time.perf_counter()
        for r in range(cpu_rows):
            try:
                omidi.decode(rows_np[r], DEFAULT_DISC.start_idx)
            except ZeroDivisionError:  # a synthetic tempo-0 token; the walk itself ran
                pass
        el = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(cpu_rows * L / el, 1), "unit": "tokens/s", "cores": 1, "kind": "port",
                               "sample": f"oracle/midi.py decode of {cpu_rows} rows x {L} tokens"}
    return out


FULL_LEN = 2000  # cfg 5: scripts/generate.py --length 2000


def decode_cached_leg(dev, rank, world, B=64, T=2048, K=32, steps=2):
    """Config 5, cached mode (a documented approximation, midiseq/generate.py):
    B=64 prompts of 2048 tokens per GPU (replicas), prefill = one exact
    forward, then one cached step per new token (KV ring of the 2048-token
    window, decode attention, skinny GEMMs, time-axis LSE over the window's
    logits ring). Steady-state rate = K new tokens per row over
    (prefill + K steps) - (prefill alone)."""
    import random
    from midiseq.generate import generate
    m = Transformer(TransformerConfig(precision="bf16", dropout=0.0)).to(dev).eval()
    src, _, meta = SyntheticMIDI(B, T, dev, rank, n_batches=1).batches[0]
    run = lambda n: generate(m, T, src, meta, num_tokens=n, rng=random.Random(0), device=dev,  # noqa: E731
                             mode="cached", return_tensor=True, group=_group(world))
    el_pre = timed(lambda: run(1), steps, 1, world, dev)
    el_all = timed(lambda: run(1 + K), steps, 1, world, dev)
    # cfg 5's own length (scripts/generate.py --length 2000): one whole run,
    # prefill included, so the window slides over every ring block
    el_full = timed(lambda: run(FULL_LEN), 1, 0, world, dev)
    cfg = m.cfg
    del m
    ms_step = (el_all - el_pre) / (steps * K) * 1e3
    # HBM bytes of one cached step: every layer's K / V ring of the
    # window (bf16), the bf16 weights once (layers + lm_head), and the
    # incremental ring LSE (msq_ring_step): per (b, v) the merged other blocks,
    # the prefix (read + write), one suffix-table entry, the new row and the
    # LSE out (22 B), plus the block entry every 64 steps amortised (32 block
    # partials, 64 rows, 64 suffix entries: ~8 B)
    d, L_, Vp, V = cfg.n_embd, cfg.n_layer, cfg.v_pad, cfg.vocab_size
    kv = L_ * B * (T + 6) * d * 2 * 2
    wts = (L_ * 12 * d * d + Vp * d) * 2
    nblk = (T + 63) // 64
    ring = B * V * (22 + (nblk * 4 + 64 * 2 + 64 * 4) / 64) + B * Vp * 2
    nbytes = kv + wts + ring
    ach = nbytes / (ms_step * 1e-3) / 1e9
    return {"value": round(world * B / (ms_step * 1e-3), 1), "unit": "new tokens/s",
            "ms_per_token_step": round(ms_step, 3), "prefill_ms": round(el_pre / steps * 1e3, 2),
            "roofline": {"kernel": "whole cached step (graph-replayed)", "bound": "hbm", "achieved": round(ach, 1),
                         "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": None,
                         "algorithmic_bytes_per_step": int(nbytes),
                         "bytes_model": "K/V ring L*B*(T+6)*d*2*2 + bf16 weights + incremental ring LSE (~30 B per (b, v)) + new row"},
            "full_length": {"new_tokens": FULL_LEN, "s": round(el_full, 3),
                            "new_tokens_per_s": round(world * B * FULL_LEN / el_full, 1)},
            "config": {"workload": "cfg 5 Transformer cached decode (KV ring, approximation of the exact window)",
                       "batch_per_gpu": B, "context": T, "new_tokens": K}}


def mamba_leg(dev, rank, world, timer, steps=3, B=8, T=4096, overlap=True, class_steps=3):
    """Config 3: models/mamba (d=1024, 10 Mamba2 layers) train step at
    T=4096, B=8 per GPU, bf16; per-class table (SSD scan on HBM bytes). With
    overlap (the engine's default two-stream backward) the class table comes
    from class_steps one-stream steps after the timed ones, as for cfg 2."""
    from midiseq.mamba import Mamba
    m = Mamba(precision="bf16").to(dev)
    m.engine.overlap_dw = overlap
    st = TrainStep(m)
    data = iter(SyntheticMIDI(B, T, dev, rank, n_batches=2))
    for _ in range(1):
        st(*next(data))
    timer.rec.clear()
    timer.on = not overlap
    el = timed(lambda: st(*next(data)), steps, 0, world, dev)
    timer.on = False
    ncls = steps
    if overlap:
        m.engine.overlap_dw = False
        ncls = max(1, class_steps)
        timer.on = True
        for _ in range(ncls):
            st(*next(data))
        torch.cuda.synchronize()
        timer.on = False
    table = timer.table(ncls)
    timer.rec.clear()
    del st, m
    tok_s = world * B * T * steps / el
    fpt = 3.0 * 174e6  # SURVEY.md §8(d) cfg 3: 174 MFLOP per token forward
    out = {"value": round(tok_s, 1), "unit": "tokens/s", "ms_per_step": round(el / steps * 1e3, 3),
           "mfu": round(tok_s / world * fpt / 1e12 / PEAK_BF16_TFLOPS, 4), "classes": table,
           "classes_source": (f"{ncls} one-stream steps after the timed ones (the timed steps run the weight-"
                              "gradient GEMMs on a second stream)") if overlap else "the timed steps (serial)",
           "config": {"workload": "cfg 3 Mamba train step (filtered CE + Adam)", "batch_per_gpu": B, "seq_len": T}}
    if "ssd_fwd" in table:
        r = table["ssd_fwd"]
        out["roofline"] = {"kernel": "SSD scan forward (msq_mamba_ssd_fwd_state: fused chunk scan + out kernels)",
                           "bound": "hbm", "achieved": r["achieved"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
                           "frac": r["frac"], "traffic": pmc_traffic("ssd_fwd", "pmc_mamba_traffic.json"),
                           "avg_launch_ms": r["avg_launch_ms"], "algorithmic_bytes": int(r["work_per_launch"]),
                           "traffic_source": "profiles/r6/pmc_mamba_traffic.json (FETCH_SIZE x2 + WRITE_SIZE passes "
                                             "of bench.py --only mamba)"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--dropout", type=float, default=0.01, help="configs/common/config.yaml values.dropout")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the decode and Mamba legs")
    ap.add_argument("--overlap", action="store_true",
                    help="weight-gradient GEMMs on a second stream: the default (kept for old command lines)")
    ap.add_argument("--serial", action="store_true",
                    help="weight-gradient GEMMs on the main stream (per-class times then sum to the step)")
    ap.add_argument("--class-steps", type=int, default=3,
                    help="with the second stream, the per-class table comes from this many extra steps "
                         "run serially after the timed ones (concurrent kernels inflate each other's times)")
    ap.add_argument("--only", choices=["mamba"], default=None,
                    help="run only the cfg 3 Mamba train leg (--steps timed steps after one warm-up; PMC passes)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU check of the launch: init gloo ranks, verify the world size, print, exit")
    args = ap.parse_args()
    # stdout carries exactly the one JSON line: everything else written to fd 1
    # (RCCL's version banner at communicator init, library chatter) goes to stderr
    out_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    def emit(obj):
        # the one line the harness parses: loop until every byte is written
        buf = memoryview((json.dumps(obj) + "\n").encode())
        while buf:
            buf = buf[os.write(out_fd, buf):]

    rank, local, world = setup_distributed(backend="gloo" if args.dry_run else None)
    assert world == args.gpus, f"bench.py --gpus {args.gpus} but the process group has {world} ranks"
    if args.dry_run:
        ranks = [None] * world
        if world > 1:
            dist.all_gather_object(ranks, rank)
            dist.destroy_process_group()
        else:
            ranks = [rank]
        if rank == 0:
            emit({"dry_run": True, "n_gpus": world, "ranks": ranks})
        return
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if args.only == "mamba":
        timer = ClassTimer()
        L.TAP = timer
        r = mamba_leg(dev, rank, world, timer, steps=args.steps, overlap=not args.serial, class_steps=args.class_steps)
        L.TAP = None
        if rank == 0:
            emit({"mamba_train": r})
        return
    cfg = TransformerConfig(n_layer=args.layers, block_len=args.seq, precision="bf16", dropout=args.dropout)
    model = Transformer(cfg).to(dev)
    overlap = not args.serial
    model.engine.overlap_dw = overlap
    step = TrainStep(model)
    data = iter(SyntheticMIDI(args.batch, args.seq, dev, rank))

    timer = ClassTimer()
    L.TAP = timer
    for _ in range(args.warmup):
        step(*next(data))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer.on = not overlap
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step(*next(data))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    timer.on = False
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    tokens = world * args.batch * args.seq * args.steps
    value = tokens / el
    ms_step = el / args.steps * 1e3
    fpt = flops_per_token(cfg, args.seq)
    if overlap:
        # per-class kernel times from serial steps: on two streams the weight-
        # gradient GEMMs share the CUs with the main stream's kernels and both
        # sides' event intervals stretch
        model.engine.overlap_dw = False
        timer.on = True
        ncls = max(1, args.class_steps)
        for _ in range(ncls):
            step(*next(data))
        torch.cuda.synchronize()
        timer.on = False
        model.engine.overlap_dw = True
        classes = timer.table(ncls)
        class_src = (f"{ncls} steps after the timed ones with the weight-gradient GEMMs on the main "
                     "stream (the timed steps run them on a second stream)")
    else:
        classes = timer.table(args.steps)
        class_src = "the timed steps (serial)"
    timer.rec.clear()
    loss_last = round(float(loss.item()), 4)

    extra = {}
    if not args.no_extra:
        del step, model
        torch.cuda.empty_cache()
        extra["decode"] = decode_leg(dev, rank, world)
        torch.cuda.empty_cache()
        extra["decode_cached"] = decode_cached_leg(dev, rank, world)
        torch.cuda.empty_cache()
        extra["mamba_train"] = mamba_leg(dev, rank, world, timer, overlap=overlap, class_steps=args.class_steps)
        torch.cuda.empty_cache()
        extra["mamba_decode"] = mamba_decode_leg(dev, rank, world)
        extra["midi_decode"] = midi_decode_leg(dev, rank, world)
    L.TAP = None
    # dominant kernel class of the train step: the largest summed time
    dom = next(k for k in classes if "frac" in classes[k])
    r = classes[dom]
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic grammar-cycled MIDI tokens, random-init weights",
            "config": {"workload": "configs/transformer default (d=1024, h=8, L=8, V=17914) train step, "
                                   f"filtered CE + Adam, dropout={args.dropout}"
                                   + (", weight-gradient GEMMs on a second stream" if overlap else
                                      ", serial backward"),
                       "model": "Transformer", "global_batch": args.batch * world, "seq_len": args.seq,
                       "parallelism": f"dp{world}"},
            "model_tflops": round(value * fpt / 1e12, 1),
            "mfu": round(value * fpt / 1e12 / (PEAK_BF16_TFLOPS * world), 4),
            "loss_last": loss_last,
            "roofline": {"kernel": f"{dom} (dominant class of the train step: {r['ms_per_step']} ms/step, "
                                   f"{r['launches_per_step']} launches/step)",
                         "bound": r["bound"], "achieved": r["achieved"], "peak": r["peak"], "unit": r["unit"],
                         "frac": r["frac"], "traffic": pmc_traffic(dom), "avg_launch_ms": r["avg_launch_ms"],
                         "algorithmic_work_per_launch": r["work_per_launch"],
                         "traffic_source": "profiles/r6/pmc_traffic.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE "
                                           "passes of this step, bytes per class launch)"},
            "classes": classes,
            "classes_source": class_src,
        }
        out.update(extra)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        emit(out)
    if dist.is_initialized():
        if world > 1:
            dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
