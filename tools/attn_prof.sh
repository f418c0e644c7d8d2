#!/bin/bash
# Attention-only GPU call: the attention parity tests (optional), then a
# rocprofv3 kernel summary of the cfg-2 relative attention fwd + bwd.
# usage: tools/attn_prof.sh <tag> [tests|notests] [env ...]
set -o pipefail
tag=${1:-attn}; shift
mode=${1:-tests}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
if [ "$mode" = "tests" ]; then
  env "$@" timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_fullsize_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/$tag/pytest.log; exit 1; }
  tail -3 gpurun_out/$tag/pytest.log
fi
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof -o run --output-format csv -- python -u tools/prof_attn.py > gpurun_out/$tag/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/$tag/prof.log; exit 1; }
f=$(ls gpurun_out/$tag/prof/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/$tag/prof/run_kernel_stats.csv)
python tools/kstat_top.py $f 14
