"""CPU-baseline calibration, run in the BUILD
container only (the reference never travels to the GPU box): the reference's
own train step (model_transformer.py + train.py filtered_logit +
CrossEntropyLoss + Adam, imported through the test-only shim of
tests/golden/make_golden.py) and the oracle restatement that bench.py times on
the box (oracle/transformer.py + oracle/loss.py + Adam), timed on the same
cores, same shapes, dropout 0:
  cfg 1   2 layers, d 128, 8 heads, T 256, B 2   
  cfg 2   default d 1024, 8 layers, 8 heads, T 2048, B 1
Writes profiles/r2/cpu_calibration.json: seconds per step of both and the
ratio restatement / reference (bench.py reports it beside cpu_baseline).

  python tools/calibrate_cpu.py [/root/reference]"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests" / "golden"))
from make_golden import RefShim  # noqa: E402
from oracle import loss as oloss, transformer as otr  # noqa: E402
from oracle.fill import REAL, grammar_tokens  # noqa: E402

OUT = REPO / "profiles" / "r2" / "cpu_calibration.json"
META = [[519, 279, 202, 202, 202, 178], [432, 277, 202, 202, 202, 173]]


def batch(B, T):
    rng = np.random.default_rng(0)
    w = np.stack([grammar_tokens(rng, REAL, T + 1) for _ in range(B)])
    return torch.from_numpy(w[:, :-1].copy()), torch.from_numpy(w[:, 1:].copy()), torch.tensor(META[:B] * (B // 2 or 1))[:B]


def time_steps(step, n):
    step()  # warm-up
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    return (time.perf_counter() - t0) / n


def reference_step(sh, hp, B, T):
    m = sh.transformer(**hp)
    m.train()
    crit = torch.nn.CrossEntropyLoss()
    opt = torch.optim.Adam(m.parameters(), lr=5e-5)
    src, trg, meta = batch(B, T)

    def step():  # train_parallel.py:174-183 without DDP
        out = m(src, meta)
        z = sh.train.filtered_logit(src, out).reshape(-1, REAL.size)
        loss = crit(z, trg.reshape(-1))
        opt.zero_grad()
        loss.backward()
        opt.step()
    return step


def oracle_step(hp, B, T):
    shapes = otr.param_shapes(hp["n_embd"], hp["n_heads"], hp["n_layer"], hp["block_len"], REAL.size, 568)
    p = {k: v.requires_grad_(True) for k, v in otr.filled_params(shapes).items()}
    opt = torch.optim.Adam(list(p.values()), lr=5e-5)
    src, trg, meta = batch(B, T)

    def step():
        loss = oloss.loss(src, trg, otr.forward(p, src, meta, hp["n_layer"], hp["n_heads"]), REAL)
        opt.zero_grad()
        loss.backward()
        opt.step()
    return step


def main(ref=Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")):
    threads = torch.get_num_threads()
    sh = RefShim(ref, REAL, 568)
    res = {"threads": threads, "host": os.uname().nodename, "configs": {}}
    for name, hp, B, T, n in (("cfg1", dict(n_embd=128, n_heads=8, n_layer=2, block_len=256), 2, 256, 10),
                              ("cfg2_b1", dict(n_embd=1024, n_heads=8, n_layer=8, block_len=2048), 1, 2048, 2)):
        r = time_steps(reference_step(sh, hp, B, T), n)
        o = time_steps(oracle_step(hp, B, T), n)
        res["configs"][name] = {"B": B, "T": T, "reference_s_per_step": round(r, 4), "oracle_s_per_step": round(o, 4),
                                "oracle_over_reference": round(o / r, 3),
                                "reference_tok_per_s": round(B * T / r, 1), "oracle_tok_per_s": round(B * T / o, 1)}
        print(name, res["configs"][name], flush=True)
    OUT.parent.mkdir(parents=True, exist_ok=True)
    OUT.write_text(json.dumps(res, indent=1) + "\n")
    print("wrote", OUT)


if __name__ == "__main__":
    main()
