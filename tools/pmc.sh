#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) over a
# command, restricted to kernels matching $1. Output: gpurun_out/pmc_<tag>/...
# Usage: tools/pmc.sh <kernel-regex> <tag> <cmd...>
set -e
re="$1"; tag="$2"; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
mkdir -p gpurun_out/pmc_$tag
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM" \
           "SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_COEXEC_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$re" -d gpurun_out/pmc_$tag/p$i -o run --output-format csv -- "$@" > gpurun_out/pmc_$tag/log$i.txt 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo ok
