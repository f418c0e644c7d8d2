#!/bin/bash
# Round-6 attention call: parity tests, kernel summary, same-box A/B against
# twin libraries. usage: tools/r6_attn.sh <tag> <libB.so> [libC.so ...]
set -o pipefail
tag=${1:-r6a}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py tests/test_fullsize_gpu.py tests/test_dropout_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/$tag/pytest.log; exit 1; }
tail -3 gpurun_out/$tag/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof -o run --output-format csv -- python -u tools/prof_attn.py > gpurun_out/$tag/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/$tag/prof.log; exit 1; }
f=$(ls gpurun_out/$tag/prof/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/$tag/prof/run_kernel_stats.csv)
python tools/kstat_top.py $f 14
for r in 1 2; do
  timeout -k 10 120 python -u tools/attn_abx.py A$r /tmp/abx A1 2>&1 | grep -v amdgpu.ids || exit 1
  i=0
  for lib in "$@"; do
    i=$((i+1))
    MSQ_LIB_PATH=$lib timeout -k 10 120 python -u tools/attn_abx.py B${i}_$r /tmp/abx A1 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
