#!/bin/bash
# HBM traffic per bench class: two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE:
# separate runs, kernel trace only, MI355X_MICROARCH.md 'HBM') over a short
# bench step, then tools/pmc_traffic.py. Usage: tools/pmc_round.sh <tag>
set -o pipefail
tag=${1:-pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/$tag/$c -o run --output-format csv -- python -u bench.py --steps 3 --warmup 0 --no-cpu-baseline --no-extra > gpurun_out/$tag/$c.log 2>&1 || { echo "pass $c failed"; tail -5 gpurun_out/$tag/$c.log; exit 1; }
done
python tools/pmc_traffic.py gpurun_out/$tag/FETCH_SIZE gpurun_out/$tag/WRITE_SIZE 3 gpurun_out/$tag/pmc_traffic.json > /dev/null && echo ok
