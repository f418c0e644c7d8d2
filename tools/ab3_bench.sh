#!/bin/bash
# Three-way same-box bench A/B of twin libraries: in-tree (B), $1 (A), $2 (C), two rounds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab3
for r in 1 2; do
  for v in B A C; do
    ev=""; [ $v = A ] && ev="MSQ_LIB_PATH=$1"; [ $v = C ] && ev="MSQ_LIB_PATH=$2"
    env $ev timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-extra > gpurun_out/ab3/$v$r.json 2> gpurun_out/ab3/$v$r.err || { echo "bench $v failed"; tail -5 gpurun_out/ab3/$v$r.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/ab3/$v$r.json'))
print('$v$r', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['classes'].items() if k.startswith('gemm')})"
  done
done
