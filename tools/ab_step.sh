#!/bin/bash
# Mamba check after a kernel change: Mamba GPU tests, the bench's Mamba leg, and a Mamba-only kernel profile.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_mamba_gpu.py tests/test_mamba_decode_gpu.py tests/test_ddp_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mt.log 2>&1; rc=$?; tail -3 gpurun_out/mt.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bm.json 2> gpurun_out/bm.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bm.json'));m=d['mamba_train'];print('train', d['ms_per_step'], 'mamba', m['ms_per_step'], {k: v['ms_per_step'] for k, v in m['classes'].items()}, m['roofline'])"
