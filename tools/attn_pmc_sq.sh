#!/bin/bash
# PMC passes (one counter set per run) over the cfg-2 attention fwd + bwd of
# tools/prof_attn.py, restricted to the kernels matching $2 (regex).
# usage: tools/attn_pmc.sh <tag> <kernel-regex> [driver.py (default tools/prof_attn.py)]
set -o pipefail
tag=${1:-attnpmc}; rx=${2:-flash_bwd}; drv=${3:-tools/prof_attn.py}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
n=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_COEXEC_CYCLES" \
           ; do
  n=$((n+1))
  MB_B=${MB_B:-32} timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$rx" -d gpurun_out/$tag/p$n -o run --output-format csv -- python -u $drv > gpurun_out/$tag/p$n.log 2>&1 || { echo "pass $n failed"; tail -20 gpurun_out/$tag/p$n.log; exit 1; }
done
python tools/pmc_sum.py gpurun_out/$tag
