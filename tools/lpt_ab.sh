#!/bin/bash
# attention / train-path GPU tests, then the train step A B A B against a twin
set -o pipefail
twin=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lpt
timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py tests/test_fullsize_gpu.py tests/test_dropout_gpu.py tests/test_transformer_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/lpt/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/lpt/pytest.log; exit 1; }
tail -1 gpurun_out/lpt/pytest.log
bash tools/ab_bench.sh lpt_step $twin notests
