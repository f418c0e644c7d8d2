#!/bin/bash
# Attention parity tests, then a same-box A/B of the attention backward key/value
# pass versions (rocprofv3 kernel summary of the cfg-2 fwd + bwd per version).
# usage: tools/attn_ab.sh <tag> [tests|notests] [versions...]
set -o pipefail
tag=${1:-attnab}; shift
mode=${1:-tests}; shift
vers=${*:-4 5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
if [ "$mode" = "tests" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py tests/test_fullsize_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/$tag/pytest.log; exit 1; }
  tail -3 gpurun_out/$tag/pytest.log
fi
for v in $vers; do
  MSQ_ATTN_BWD_KV=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof_kv$v -o run --output-format csv -- python -u tools/prof_attn.py > gpurun_out/$tag/prof_kv$v.log 2>&1 || { echo "rocprof kv$v failed"; tail -20 gpurun_out/$tag/prof_kv$v.log; exit 1; }
  f=$(ls gpurun_out/$tag/prof_kv$v/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/$tag/prof_kv$v/run_kernel_stats.csv)
  echo "== kv$v"; python tools/kstat_top.py $f 10
done
