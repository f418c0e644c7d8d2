"""Data-parallel step on the GPU through the real engine:
two ranks on the one leased GPU (gloo over CUDA tensors; RCCL needs one GPU
per rank) run tests/ddp_worker.py — TrainStep with the backward's per-layer
bucket hooks, the weight-gradient side stream and the all-reduce side stream
— and are compared with a single process running the same TrainStep.

* "same": both ranks get the same 2 sequences. Their SUM all-reduce divided
  by world is then exactly the single-process gradient of those sequences
  (x + x = 2x in fp32): a bucket that is never reduced, reduced twice, or
  reduced before the dW stream wrote it shows up far above the tolerance
  (fp32 atomics in the embedding backward: 1e-5 relative).
* "split": the ranks get sequences 0-1 and 2-3; the averaged gradient equals
  the single-process gradient of all 4 (the loss is a mean over B*T) up to
  bf16 summation order.
Reference loop: train_parallel.py:143-183 (DDP ctor broadcast, backward
all-reduce, Adam)."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = Path(__file__).parent


def _run_world2(kind, mode, tmp_path, env=None, nproc=2):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tmp_path / f"{kind}_{mode}_{len(env or {})}.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(HERE / "ddp_worker.py"), kind, mode, str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, OMP_NUM_THREADS="4", **(env or {})))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return np.load(out)


def _single(kind, rows):
    sys.path.insert(0, str(HERE))
    import ddp_worker as w
    from midiseq.train_parallel import TrainStep
    model = w.build_model(kind).to("cuda")
    step = TrainStep(model)
    src, trg, meta = w.full_batch()
    loss = step(src[rows].cuda(), trg[rows].cuda(), meta[rows].cuda())
    torch.cuda.synchronize()
    return step.grads.cpu().numpy(), model.flat.data.cpu().numpy(), loss.item()


@pytest.mark.parametrize("kind", ["transformer", "mamba"])
def test_world2_same_data_equals_single_process(kind, tmp_path):
    got = _run_world2(kind, "same", tmp_path)
    g, flat, loss = _single(kind, slice(0, 2))
    assert abs(float(got["loss"]) - loss) <= 1e-5 * abs(loss)
    err = np.abs(got["grads"] - g).max()
    print(f"\n{kind} same-data max |grad diff| = {err:.3e} (max |g| {np.abs(g).max():.3e})")
    assert err <= 1e-5 * np.abs(g).max(), err
    # parameters after one Adam step (scale 1/world folded into the kernel).
    # Step 1 of Adam moves each parameter by lr * g / (|g| + eps): where |g| is
    # near eps (1e-8) the 1e-5-relative atomics noise of the gradient shows,
    # so allow a few elements up to 2 % of lr (5e-5)
    d = np.abs(got["flat"] - flat)
    assert d.max() <= 1e-6 and (d > 2e-7).sum() <= 16, (d.max(), (d > 2e-7).sum())


@pytest.mark.parametrize("kind", ["transformer", "mamba"])
def test_world2_split_batch_averages_gradients(kind, tmp_path):
    got = _run_world2(kind, "split", tmp_path)
    g, _, _ = _single(kind, slice(0, 4))
    a, b = got["grads"].astype(np.float64), g.astype(np.float64)
    nr = np.linalg.norm(a - b) / np.linalg.norm(b)
    cos = float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b)))
    assert nr < 2e-2 and cos > 0.9995, (nr, cos)


@pytest.mark.parametrize("kind", ["transformer", "mamba"])
def test_world2_per_bucket_adam_equals_global_adam(kind, tmp_path):
    """The per-bucket Adam (run on the all-reduce side stream as each bucket's
    SUM arrives, TrainStep default) gives, from the same start and the same
    reduced gradients, the parameters and moments of one global Adam after the
    backward (the MSQ_GLOBAL_ADAM=1 update) bit for bit: the update is
    elementwise and the buckets tile the flat buffer. (Two separate runs are
    not compared: the backward's atomics make their gradients differ in the
    last bits.) The MSQ_GLOBAL_ADAM=1 path itself must also run and agree to
    within that gradient noise."""
    a = _run_world2(kind, "bucketcheck", tmp_path)
    assert np.array_equal(a["flat"], a["ref"])
    assert np.array_equal(a["m"], a["m_ref"]) and np.array_equal(a["v"], a["v_ref"])
    b = _run_world2(kind, "split", tmp_path, env={"MSQ_GLOBAL_ADAM": "1"})
    d = np.abs(a["flat"] - b["flat"])
    assert d.max() <= 1e-6 and (d > 2e-7).sum() <= 16, (d.max(), (d > 2e-7).sum())


@pytest.mark.parametrize("kind", ["transformer", "mamba"])
def test_rccl_world1_bucket_path(kind, tmp_path):
    """The RCCL path itself: torch.distributed.run with one
    rank, setup_distributed() -> backend nccl (= RCCL), TrainStep(ddp=True):
    every layer bucket is a ProcessGroupNCCL all_reduce issued from the side
    stream, waited on that stream, then the per-bucket Adam there. After two
    steps the parameters and moments equal one global Adam over the same
    reduced gradients bit for bit (a bucket whose Adam ran before its
    collective, or never, or twice, breaks this), and the gradients equal a
    bucket-free TrainStep's up to the backward's atomics noise.
    Reference: train_parallel.py:144-151 (init_process_group nccl, DDP)."""
    a = _run_world2(kind, "rccl1", tmp_path, nproc=1, env={"MSQ_DDP_BUCKETS": "1"} if kind == "mamba" else None)
    assert str(a["backend"]) == "nccl"
    assert np.array_equal(a["flat"], a["ref"])
    assert np.array_equal(a["m"], a["m_ref"]) and np.array_equal(a["v"], a["v_ref"])
    g, gp = a["grads"], a["grads_plain"]
    err = np.abs(g - gp).max()
    assert err <= 1e-5 * np.abs(gp).max(), err
    assert abs(float(a["loss"]) - float(a["loss_plain"])) <= 1e-5 * abs(float(a["loss_plain"]))
    d = np.abs(a["flat"] - a["flat_plain"])
    assert d.max() <= 2e-6 and (d > 2e-7).sum() <= 32, (d.max(), (d > 2e-7).sum())
