#!/bin/bash
# Full GPU suite, then (unless the suite crashed) the attention kernel summary
# and same-box A/B against twin libraries. usage: tools/r6_full.sh <tag> [libB.so ...]
set -o pipefail
tag=${1:-r6f}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/$tag/pytest.log; grep -E "FAILED|ERROR" gpurun_out/$tag/pytest.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof -o run --output-format csv -- python -u tools/prof_attn.py > gpurun_out/$tag/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/$tag/prof.log; exit 1; }
f=$(ls gpurun_out/$tag/prof/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/$tag/prof/run_kernel_stats.csv)
python tools/kstat_top.py $f 10
for r in 1 2; do
  timeout -k 10 120 python -u tools/attn_abx.py A$r /tmp/abx A1 2>&1 | grep -v amdgpu.ids || exit 1
  i=0
  for lib in "$@"; do
    i=$((i+1))
    MSQ_LIB_PATH=$lib timeout -k 10 120 python -u tools/attn_abx.py B${i}_$r /tmp/abx A1 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
exit $rc
