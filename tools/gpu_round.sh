#!/bin/bash
# One GPU call: parity tests, bench line, rocprofv3 kernel stats of the bench
# (weight-gradient GEMMs on a second stream - the default - and serial, whose
# kernel durations the bench's class table matches). Usage: tools/gpu_round.sh <tag> [skip-tests]
set -o pipefail
tag=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$tag/pytest.log; exit 1; }
  tail -3 gpurun_out/$tag/pytest.log
fi
timeout -k 10 600 python -u bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || { echo "bench failed"; tail -30 gpurun_out/$tag/bench.err; exit 1; }
cat gpurun_out/$tag/bench.json
timeout -k 10 300 python -u bench.py --serial --no-extra --no-cpu-baseline --steps 5 > gpurun_out/$tag/bench_serial.json 2> gpurun_out/$tag/bench_serial.err || { echo "serial bench failed"; tail -20 gpurun_out/$tag/bench_serial.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof -o run --output-format csv -- python -u bench.py --serial --steps 5 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/$tag/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/$tag/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof_overlap -o run --output-format csv -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/$tag/prof_overlap.log 2>&1 || { echo "rocprof overlap failed"; tail -20 gpurun_out/$tag/prof_overlap.log; exit 1; }
echo done
