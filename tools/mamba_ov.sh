#!/bin/bash
# Mamba two-stream backward: its GPU tests (+ the Transformer's and DDP's, which
# share ops.SideStream), then same-box A/B of the Mamba train step
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mov
true || timeout -k 10 500 python -u -m pytest tests/test_mamba_gpu.py tests/test_transformer_gpu.py tests/test_ddp_gpu.py tests/test_decode_attn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mov/tests.log 2>&1; rc=$?; tail -4 gpurun_out/mov/tests.log; [ $rc = 0 ] || exit 1
bash tools/mamba_ab.sh "A=1 -- --serial" "A=0"
