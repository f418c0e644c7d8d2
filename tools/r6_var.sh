#!/bin/bash
# Kernel time of one kernel (regex) under each library (rocprofv3 --stats over
# tools/prof_attn.py), then optional PMC passes of the in-tree library.
# usage: tools/r6_var.sh <tag> <kernel-regex> <pmc|nopmc> lib1.so [lib2.so ...]  ("-" = in-tree)
set -o pipefail
tag=$1; rx=$2; pmc=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
i=0
for lib in "$@"; do
  i=$((i+1))
  if [ "$lib" = "-" ]; then envs=""; else envs="MSQ_LIB_PATH=$lib"; fi
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/v$i -o run --output-format csv -- python -u tools/prof_attn.py > gpurun_out/$tag/v$i.log 2>&1 || { echo "rocprof $lib failed"; tail -20 gpurun_out/$tag/v$i.log; exit 1; }
  f=$(ls gpurun_out/$tag/v$i/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/$tag/v$i/run_kernel_stats.csv)
  echo "== $lib"; python tools/kstat_top.py $f 30 | grep -E "$rx"
done
if [ "$pmc" = "pmc" ]; then
  n=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
             "SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_COEXEC_CYCLES" \
             "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    n=$((n+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$rx" -d gpurun_out/$tag/p$n -o run --output-format csv -- python -u tools/prof_attn.py > gpurun_out/$tag/p$n.log 2>&1 || { echo "pass $n failed"; tail -20 gpurun_out/$tag/p$n.log; exit 1; }
  done
  python tools/pmc_sum.py gpurun_out/$tag
fi
