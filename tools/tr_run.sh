cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "transpose or gemm" > gpurun_out/tr_test.log 2>&1 || { tail -30 gpurun_out/tr_test.log; exit 1; }
tail -1 gpurun_out/tr_test.log
bash tools/ab_mamba.sh tr1 /root/repo/ab_head.so
