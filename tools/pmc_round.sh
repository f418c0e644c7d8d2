#!/bin/bash
# HBM traffic per bench class: two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE:
# separate runs, kernel trace only, MI355X_MICROARCH.md 'HBM') over a short
# bench step, then tools/pmc_traffic.py; the same for the Mamba train step
# (bench.py --only mamba: one warm-up + 3 timed + 3 one-stream class steps = 7 profiled steps).
# Usage: tools/pmc_round.sh <tag> [train|mamba|both]
set -o pipefail
tag=${1:-pmc}
which=${2:-both}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
if [ "$which" != mamba ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/$tag/$c -o run --output-format csv -- python -u bench.py --serial --steps 3 --warmup 0 --no-cpu-baseline --no-extra > gpurun_out/$tag/$c.log 2>&1 || { echo "pass $c failed"; tail -5 gpurun_out/$tag/$c.log; exit 1; }
  done
  python tools/pmc_traffic.py gpurun_out/$tag/FETCH_SIZE gpurun_out/$tag/WRITE_SIZE 3 gpurun_out/$tag/pmc_traffic.json > /dev/null && echo train ok || exit 1
fi
if [ "$which" != train ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/$tag/m_$c -o run --output-format csv -- python -u bench.py --only mamba --steps 3 --no-cpu-baseline > gpurun_out/$tag/m_$c.log 2>&1 || { echo "mamba pass $c failed"; tail -5 gpurun_out/$tag/m_$c.log; exit 1; }
  done
  python tools/pmc_traffic.py gpurun_out/$tag/m_FETCH_SIZE gpurun_out/$tag/m_WRITE_SIZE 7 gpurun_out/$tag/pmc_mamba_traffic.json mamba > /dev/null && echo mamba ok || exit 1
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/m_prof -o run --output-format csv -- python -u bench.py --only mamba --steps 3 --no-cpu-baseline > gpurun_out/$tag/m_prof.log 2>&1 || { echo "mamba stats failed"; exit 1; }
fi
echo done
