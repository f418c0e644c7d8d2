#!/bin/bash
# the whole GPU suite, then the train step A (twin) B (tree) A B
set -o pipefail
twin=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fab
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fab/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/fab/pytest.log; exit 1; }
tail -1 gpurun_out/fab/pytest.log
bash tools/ab_bench.sh fab_step $twin notests
