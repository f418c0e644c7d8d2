#!/bin/bash
# Same-box A/B: attention dropout masks on a side stream (MSQ_MASK_SIDE=1) vs in the layer loop.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
MSQ_MASK_SIDE=1 timeout -k 10 400 python -u -m pytest tests/test_transformer_gpu.py tests/test_dropout_gpu.py tests/test_ddp_gpu.py tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ms.log 2>&1; rc=$?; tail -2 gpurun_out/ms.log; [ $rc = 0 ] || exit 1
run() { tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/ab_$tag.json 2>gpurun_out/ab.err || return 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));c=d['classes'];print('$tag', d['ms_per_step'], d['loss_last'])"
}
run base A=1 && run side MSQ_MASK_SIDE=1 && run base2 A=1 && run side2 MSQ_MASK_SIDE=1
