#!/bin/bash
# Mamba step kernel summary (rocprofv3 --stats over bench.py --only mamba) and
# SQ / traffic counter passes of one kernel. usage: tools/r6_mpmc.sh <tag> <kernel-regex>
set -o pipefail
tag=${1:-r6mp}; rx=${2:-grad_kernel}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof -o run --output-format csv -- python -u bench.py --only mamba --steps 5 --no-cpu-baseline > gpurun_out/$tag/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/$tag/prof.log; exit 1; }
f=$(ls gpurun_out/$tag/prof/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/$tag/prof/run_kernel_stats.csv)
python tools/kstat_top.py $f 12
n=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_COEXEC_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$rx" -d gpurun_out/$tag/p$n -o run --output-format csv -- python -u bench.py --only mamba --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$tag/p$n.log 2>&1 || { echo "pass $n failed"; tail -20 gpurun_out/$tag/p$n.log; exit 1; }
done
python tools/pmc_sum.py gpurun_out/$tag
