#!/bin/bash
# Round-5 GPU call: GPU suite, default bench line, and the bench under
# torch.distributed.run with one rank over RCCL (bucket path forced on).
# Usage: tools/gpu_r5.sh <tag> [skip-tests]
set -o pipefail
tag=${1:-r5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/$tag/pytest.log; exit 1; }
  tail -3 gpurun_out/$tag/pytest.log
fi
timeout -k 10 600 python -u bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || { echo "bench failed"; tail -30 gpurun_out/$tag/bench.err; exit 1; }
cat gpurun_out/$tag/bench.json
MSQ_DDP_BUCKETS=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29531 bench.py --gpus 1 --no-extra --no-cpu-baseline > gpurun_out/$tag/bench_rccl1.json 2> gpurun_out/$tag/bench_rccl1.err || { echo "rccl bench failed"; tail -30 gpurun_out/$tag/bench_rccl1.err; exit 1; }
grep "^{" gpurun_out/$tag/bench_rccl1.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rccl1', d['ms_per_step'], d['value'])"
echo done
