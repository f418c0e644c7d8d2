#!/bin/bash
# loss-path GPU tests, then the train step A B A B against a twin (tools/ab_bench.sh)
set -o pipefail
twin=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lossab
timeout -k 10 500 python -u -m pytest tests/test_transformer_gpu.py tests/test_fullsize_gpu.py tests/test_head_stats_gpu.py tests/test_batch32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lossab/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/lossab/pytest.log; exit 1; }
tail -1 gpurun_out/lossab/pytest.log
bash tools/ab_bench.sh lossab_step $twin notests
