"""Pins the CPU Mamba oracle (sequential-recurrence restatement) against G5:
the reference's own models/mamba/mamba.py run with HF transformers' pure-torch
Mamba2 mixer standing in for mamba_ssm.Mamba2 (tests/golden/make_golden.py)."""
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import loss as oloss
from oracle import mamba2 as om
from oracle.fill import REAL, hash_uniform
from golden_check import check_grad

G = Path(__file__).parent / "golden"


def test_default_param_count_matches_reference_notebook():
    g5 = np.load(G / "g5_mamba.npz")
    shapes = om.param_shapes(1024, 10, REAL.size, 568)
    n = sum(int(np.prod(s)) for s in shapes.values())
    assert n == int(g5["default_param_count"]) == 101_972_666  # scripts/Test Accuracy.ipynb:52


@pytest.mark.parametrize("chunked", [False, True])
def test_mamba_fwd_bwd_matches_golden(chunked):
    """Both oracle forms (sequential recurrence; chunked SSD with Q = 256, which
    T = 300 (+6 meta) crosses) against the reference's outputs."""
    g5 = np.load(G / "g5_mamba.npz")
    shapes = om.param_shapes(128, 2, REAL.size, 568)
    p = {k: v.requires_grad_(True) for k, v in om.filled_params(shapes).items()}
    src, trg, meta = (torch.from_numpy(g5[n]) for n in ("src", "trg", "meta"))
    logits = om.forward(p, src, meta, 2, chunked=chunked)
    loss = oloss.loss(src, trg, logits, REAL)
    loss.backward()
    assert abs(loss.item() - float(g5["loss"])) < 1e-4 * abs(float(g5["loss"]))
    P = torch.from_numpy(hash_uniform(REAL.size * 8, 7).reshape(REAL.size, 8).astype(np.float32))
    np.testing.assert_allclose((logits.detach() @ P).numpy(), g5["logits_proj"], rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(logits.detach()[:, [0, 149, 299]].numpy(), g5["logits_rows"], rtol=1e-4, atol=1e-4)
    for k, t in p.items():
        if k in ("norm.bias", "output_layer.bias"):  # analytically zero (shift invariance along T)
            assert t.grad.abs().max().item() < 1e-4 * p["output_layer.weight"].grad.abs().max().item(), k
            continue
        check_grad(k, t.grad.numpy(), g5[f"gsum:{k}"], g5[f"gpick:{k}"], 2e-3)
