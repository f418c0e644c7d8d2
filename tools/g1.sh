cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/g1
timeout -k 10 300 python -u tools/gemm_square.py > gpurun_out/g1/square.txt 2>&1 && timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/g1/bench.txt 2>&1; cat gpurun_out/g1/square.txt gpurun_out/g1/bench.txt | grep -v amdgpu.ids
