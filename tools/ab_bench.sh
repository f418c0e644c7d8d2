#!/bin/bash
# GPU tests on the in-tree build, then the cfg-2 train step (bench.py, no CPU
# baseline / extra legs) A, B, A, B with A = MSQ_LIB_PATH=$2 (a tools/build_ab.sh twin).
# usage: tools/ab_bench.sh <tag> <twin.so> [tests|notests]
set -o pipefail
tag=$1; twin=$2; mode=${3:-tests}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
if [ "$mode" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$tag/pytest.log; exit 1; }
  tail -1 gpurun_out/$tag/pytest.log
fi
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then ev="MSQ_LIB_PATH=$twin"; else ev=""; fi
    env $ev timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-extra > gpurun_out/$tag/$v$r.json 2> gpurun_out/$tag/$v$r.err || { echo "bench $v failed"; tail -5 gpurun_out/$tag/$v$r.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/$tag/$v$r.json'))
print('$v$r' + (' (twin)' if '$v' == 'A' else ' (tree)'), d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['classes'].items() if v['ms_per_step'] > 1.0})"
  done
done
