#!/bin/bash
# Mamba GPU tests on the in-tree library, then the Mamba train step A B A B
# against a library file (MSQ_LIB_PATH). usage: tools/mamba_abl.sh <tag> <libB.so> [tests|notests]
set -o pipefail
tag=$1; lib=$2; mode=${3:-tests}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
if [ "$mode" = tests ]; then
  timeout -k 10 400 python -u -m pytest tests/test_mamba_gpu.py tests/test_mamba_decode_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$tag/pytest.log; exit 1; }
  tail -1 gpurun_out/$tag/pytest.log
fi
for r in 1 2; do
  for v in A B; do
    if [ $v = B ]; then export MSQ_LIB_PATH=$lib; else unset MSQ_LIB_PATH; fi
    timeout -k 10 200 python -u bench.py --only mamba --steps 5 --no-cpu-baseline > gpurun_out/$tag/$v$r.json 2> gpurun_out/$tag/$v$r.err || { echo "bench $v failed"; tail -5 gpurun_out/$tag/$v$r.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/$tag/$v$r.json')); m=d.get('mamba_train', d)
print('$v$r', m.get('ms_per_step'), {k: v['ms_per_step'] for k, v in m.get('classes', {}).items() if k.startswith('ssd') or k.startswith('mamba')})"
  done
done
