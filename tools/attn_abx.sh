#!/bin/bash
# Same-box A/B of attention libraries with dropout on (tools/attn_abx.py):
# A = the in-tree libmidiseq.so, B.. = the given .so files; rounds A B A B.
# Optionally runs the attention GPU tests against the in-tree library first.
# usage: tools/attn_abx.sh <tag> [tests|notests] <libB.so> [libC.so ...]
set -o pipefail
tag=${1:-abx}; shift
mode=${1:-notests}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
if [ "$mode" = "tests" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py tests/test_fullsize_gpu.py tests/test_dropout_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/$tag/pytest.log; exit 1; }
  tail -3 gpurun_out/$tag/pytest.log
fi
for r in 1 2; do
  timeout -k 10 120 python -u tools/attn_abx.py A$r /tmp/abx A1 2>&1 | grep -v amdgpu.ids || exit 1
  i=0
  for lib in "$@"; do
    i=$((i+1))
    MSQ_LIB_PATH=$lib timeout -k 10 120 python -u tools/attn_abx.py B${i}_$r /tmp/abx A1 2>&1 | grep -v amdgpu.ids || exit 1
  done
done

