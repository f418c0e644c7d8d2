"""Sharded decode (generate(..., group=...)): two ranks on
the one leased GPU (gloo) each decode half of a 4-prompt batch; their rows
must equal, bit for bit, the rows of ONE process decoding all 4 with the same
Python RNG (the k choice replayed over every global row on every rank: one
all-gather of the last tokens per step), the same recorded uniforms (sliced
by global row) and the same torch seed (device uniforms drawn for all rows,
then sliced). fp32 engine, exact and cached modes. Reference loop:
scripts/generate.py:34-85."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = Path(__file__).parent


@pytest.mark.parametrize("mode", ["exact", "cached"])
def test_world2_decode_rows_equal_single_process(mode, tmp_path):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tmp_path / mode
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(HERE / "decode_shard_worker.py"), mode, str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=dict(os.environ, OMP_NUM_THREADS="4"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    parts = [np.load(f"{out}_{k}.npz") for k in range(2)]
    sys.path.insert(0, str(HERE))
    import decode_shard_worker as w
    model = w.build_model()
    src, meta, us = w.prompts()
    a, b = w.run(model, src, meta, mode, us)
    np.testing.assert_array_equal(np.concatenate([p["a"] for p in parts]), a)
    np.testing.assert_array_equal(np.concatenate([p["b"] for p in parts]), b)
    assert not np.array_equal(a[:, w.T0:], b[:, w.T0:])  # the two RNG paths really differ
