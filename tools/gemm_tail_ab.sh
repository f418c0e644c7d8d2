#!/bin/bash
# GEMM / train-path GPU tests, tools/gemm_tail.py A (tree) / B (twin) twice,
# then the train step A B A B (tools/ab_bench.sh). usage: tools/gemm_tail_ab.sh <twin.so>
set -o pipefail
twin=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gtail
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py tests/test_fullsize_gpu.py tests/test_decode_cached_gpu.py tests/test_batch32_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/gtail/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/gtail/pytest.log; exit 1; }
tail -1 gpurun_out/gtail/pytest.log
for r in 1 2; do
  timeout -k 10 200 python -u tools/gemm_tail.py A$r /tmp/gt $( [ $r = 2 ] && echo A1 ) 2>&1 | grep -v amdgpu.ids || exit 1
  MSQ_LIB_PATH=$twin timeout -k 10 200 python -u tools/gemm_tail.py B$r /tmp/gt A1 2>&1 | grep -v amdgpu.ids || exit 1
done
bash tools/ab_bench.sh gtail_step $twin notests
