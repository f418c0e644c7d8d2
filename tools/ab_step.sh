#!/bin/bash
# Adam kernel check: optimizer / DDP GPU tests, then the bench's adam class (two runs).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/at.log 2>&1; rc=$?; tail -2 gpurun_out/at.log; [ $rc = 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/ad$i.json 2>gpurun_out/ad.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ad$i.json'));c=d['classes'];print(d['ms_per_step'], 'adam', c['adam'])"
done
