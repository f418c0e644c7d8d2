#!/bin/bash
# Decode-step A/B in one call: the decode GPU tests on the in-tree build, then
# tools/decode_prof.py (Mamba and Transformer) A, B, A, B with
# A = MSQ_LIB_PATH=$2 (a tools/build_ab.sh twin).  usage: tools/ab_decode.sh <tag> <twin.so>
set -o pipefail
tag=$1; twin=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests/test_mamba_decode_gpu.py tests/test_decode_cached_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$tag/pytest.log; exit 1; }
tail -1 gpurun_out/$tag/pytest.log
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then ev="${AB_ENV:-MSQ_LIB_PATH=$twin}"; else ev=""; fi
    for k in mamba transformer; do
      env $ev timeout -k 10 200 python -u tools/decode_prof.py $k 100 > gpurun_out/$tag/$v$r$k.log 2>&1 || { echo "$v $k failed"; tail -5 gpurun_out/$tag/$v$r$k.log; exit 1; }
      echo "$v$r $k: $(grep -h 'step\|iteration' gpurun_out/$tag/$v$r$k.log | tr '\n' ' ')"
    done
  done
done
