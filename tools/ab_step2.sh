#!/bin/bash
# Same-box A/B of the cfg-2 train step: A = the in-tree library with the
# default environment, B = the given env assignments (e.g. MSQ_LIB_PATH=...);
# rounds A B A B, the step time and the class times that moved.
# usage: tools/ab_step2.sh <tag> [tests] VAR=VALUE ...
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
if [ "$1" = tests ]; then
  shift
  timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_head_stats_gpu.py tests/test_transformer_gpu.py tests/test_train_gpu.py tests/test_fullsize_gpu.py tests/test_generate_gpu.py tests/test_decode_cached_gpu.py tests/test_mamba_decode_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$tag/pytest.log; exit 1; }
  tail -1 gpurun_out/$tag/pytest.log
fi
run() { v=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/$tag/$v.json 2> gpurun_out/$tag/$v.err || { echo "bench $v failed"; tail -5 gpurun_out/$tag/$v.err; return 1; }
  python -c "
import json; d=json.load(open('gpurun_out/$tag/$v.json')); c=d['classes']
print('$v', d['ms_per_step'], d['loss_last'], {k: c[k]['ms_per_step'] for k in ('gemm_fwd', 'gemm_dX', 'gemm_dW', 'loss', 'attn_fwd', 'attn_bwd') if k in c})"
}
run A1 A=1 && run B1 "$@" && run A2 A=1 && run B2 "$@"
