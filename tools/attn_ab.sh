#!/bin/bash
# Attention parity tests, then a same-box A/B of environment settings
# (rocprofv3 kernel summary of the cfg-2 fwd + bwd per setting; "base" = none).
# usage: tools/attn_ab.sh <tag> [tests|notests] [base | VAR=value ...]
set -o pipefail
tag=${1:-attnab}; shift
mode=${1:-tests}; shift
vers=${*:-base}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
if [ "$mode" = "tests" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py tests/test_fullsize_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/$tag/pytest.log; exit 1; }
  tail -3 gpurun_out/$tag/pytest.log
fi
for v in $vers; do
  n=${v//[^A-Za-z0-9]/_}
  ev=""; [ "$v" != base ] && ev="$v"
  env $ev timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof_$n -o run --output-format csv -- python -u tools/prof_attn.py > gpurun_out/$tag/prof_$n.log 2>&1 || { echo "rocprof $v failed"; tail -20 gpurun_out/$tag/prof_$n.log; exit 1; }
  f=$(ls gpurun_out/$tag/prof_$n/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/$tag/prof_$n/run_kernel_stats.csv)
  echo "== $v"; python tools/kstat_top.py $f 10
done
