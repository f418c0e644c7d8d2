#!/bin/bash
# Same-box attention A/B only (no tests): tools/attn_abx.py on the in-tree
# library (A) and each twin, two rounds. usage: tools/abx_libs.sh lib1.so [lib2.so ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in ${ABX_ROUNDS:-1 2}; do
  timeout -k 10 120 python -u tools/attn_abx.py A$r /tmp/abx A1 2>&1 | grep -v amdgpu.ids || exit 1
  i=0
  for lib in "$@"; do
    i=$((i+1))
    MSQ_LIB_PATH=$lib timeout -k 10 120 python -u tools/attn_abx.py B${i}_$r /tmp/abx A1 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
