#!/bin/bash
# rocprofv3 kernel summaries of the cfg-2 train step (one-stream and the timed
# two-stream form) and the PMC traffic passes (tools/pmc_round.sh).
# Usage: tools/prof_r5.sh <tag>
set -o pipefail
tag=${1:-r5prof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/serial -o run --output-format csv -- python -u bench.py --serial --steps 7 --no-cpu-baseline --no-extra > gpurun_out/$tag/serial.log 2>&1 || { echo "serial stats failed"; tail -5 gpurun_out/$tag/serial.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/overlap -o run --output-format csv -- python -u bench.py --steps 7 --no-cpu-baseline --no-extra > gpurun_out/$tag/overlap.log 2>&1 || { echo "overlap stats failed"; tail -5 gpurun_out/$tag/overlap.log; exit 1; }
bash tools/pmc_round.sh $tag both
