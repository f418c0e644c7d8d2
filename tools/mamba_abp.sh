#!/bin/bash
# rocprofv3 kernel summaries of the Mamba train step for the in-tree library
# (A) and a library file (B). usage: tools/mamba_abp.sh <tag> <libB.so>
set -o pipefail
tag=$1; lib=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
for v in A B; do
  if [ $v = B ]; then export MSQ_LIB_PATH=$lib; else unset MSQ_LIB_PATH; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/p_$v -o run --output-format csv -- python -u bench.py --only mamba --steps 3 --no-cpu-baseline > gpurun_out/$tag/p_$v.log 2>&1 || { echo "rocprof $v failed"; tail -5 gpurun_out/$tag/p_$v.log; exit 1; }
  f=$(ls gpurun_out/$tag/p_$v/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/$tag/p_$v/run_kernel_stats.csv)
  echo "== $v"; python tools/kstat_top.py $f 14
done
