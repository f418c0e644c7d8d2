#!/bin/bash
# Mamba decode: fused in_proj + conv step (default) vs the two-launch path (MSQ_NO_CONV_FUSE=1).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_mamba_decode_gpu.py tests/test_generate_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dect.log 2>&1; rc=$?; tail -3 gpurun_out/dect.log; [ $rc = 0 ] || exit 1
for v in fused two fused two; do
  if [ $v = two ]; then export MSQ_NO_CONV_FUSE=1; else unset MSQ_NO_CONV_FUSE; fi
  echo "== $v"; timeout -k 10 120 python -u tools/decode_prof.py mamba 60 2>&1 | grep -v amdgpu.ids | tail -4 || exit 1
done
