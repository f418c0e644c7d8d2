#!/bin/bash
# GEMM split-K reduction check: DDP / transformer GPU tests (bitwise paths), then the reduce kernel's rocprof time.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lt.log 2>&1; rc=$?; tail -3 gpurun_out/lt.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pk -o run --output-format csv -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/pk.log 2>&1 || exit 1
grep -h "splitk_reduce\|gemm256_kernel<1, 1, 5" gpurun_out/pk/run_kernel_stats.csv | cut -c1-160
