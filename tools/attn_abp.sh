#!/bin/bash
# rocprofv3 kernel summaries of tools/attn_abx.py (cfg-2 attention with
# dropout) for the in-tree library (A) and each given library (B1, B2, ...).
# usage: tools/attn_abp.sh <tag> <libB.so> [libC.so ...]
set -o pipefail
tag=${1:-abp}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
run() {  # name, lib
  if [ -n "$2" ]; then export MSQ_LIB_PATH=$2; else unset MSQ_LIB_PATH; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/p_$1 -o run --output-format csv -- python -u tools/attn_abx.py $1 /tmp/abp > gpurun_out/$tag/p_$1.log 2>&1 || { echo "rocprof $1 failed"; tail -20 gpurun_out/$tag/p_$1.log; exit 1; }
  f=$(ls gpurun_out/$tag/p_$1/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/$tag/p_$1/run_kernel_stats.csv)
  echo "== $1 ${2:-in-tree}"; python tools/kstat_top.py $f 8
}
run A ""
i=0
for lib in "$@"; do i=$((i+1)); run B$i $lib; done
