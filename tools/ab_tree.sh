#!/bin/bash
# A/B of a whole source tree: A = the copy in _abtree/ (git archive of a
# revision + its built libmidiseq.so), B = this tree; Mamba GPU tests on B,
# then the Mamba train step A B A B.  usage: tools/ab_tree.sh <tag>
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests/test_mamba_gpu.py tests/test_mamba_decode_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$tag/pytest.log; exit 1; }
tail -1 gpurun_out/$tag/pytest.log
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then d=_abtree; else d=.; fi
    (cd $d && timeout -k 10 200 python -u bench.py --only mamba --steps 5 --no-cpu-baseline) > gpurun_out/$tag/$v$r.json 2> gpurun_out/$tag/$v$r.err || { echo "bench $v failed"; tail -5 gpurun_out/$tag/$v$r.err; exit 1; }
    python -c "
import json,sys; d=json.load(open('gpurun_out/$tag/$v$r.json')); m=d.get('mamba_train', d)
print('$v$r', m.get('ms_per_step'), {k: v['ms_per_step'] for k, v in m.get('classes', {}).items() if k.startswith('ssd') or k.startswith('mamba')})"
  done
done
