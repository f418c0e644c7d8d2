#!/bin/bash
# LayerNorm backward alone: timing (queue / ordered) and PMC passes of the queue form.
set -o pipefail
tag=${1:-r6ln}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
# A/B against a twin library (second argument) when given: A B A B
for r in 1 2; do
  if [ -n "$2" ]; then
    echo -n "A(twin) "; MSQ_LIB_PATH=$2 timeout -k 10 120 python -u tools/ln_only.py queue 20 || exit 1
    echo -n "A(twin) "; MSQ_LIB_PATH=$2 timeout -k 10 120 python -u tools/ln_only.py ordered 20 || exit 1
  fi
  echo -n "B(tree) "; timeout -k 10 120 python -u tools/ln_only.py queue 20 || exit 1
  echo -n "B(tree) "; timeout -k 10 120 python -u tools/ln_only.py ordered 20 || exit 1
done
[ "$3" = "nopmc" ] && exit 0
n=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_COEXEC_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "ln_bwd|ln_reduce" -d gpurun_out/$tag/p$n -o run --output-format csv -- python -u tools/ln_only.py queue 3 > gpurun_out/$tag/p$n.log 2>&1 || { echo "pass $n failed"; tail -20 gpurun_out/$tag/p$n.log; exit 1; }
done
python tools/pmc_sum.py gpurun_out/$tag
