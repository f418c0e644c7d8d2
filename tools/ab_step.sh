#!/bin/bash
# Same-box A/B of the SSD decode-step state mapping (MSQ_SSD_STEP_ROWS=1: the previous one).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in new rows; do
  if [ $v = rows ]; then export MSQ_SSD_STEP_ROWS=1; else unset MSQ_SSD_STEP_ROWS; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pss_$v -o run --output-format csv -- python -u tools/decode_prof.py mamba 40 > gpurun_out/pss_$v.log 2>&1 || exit 1
  echo "== $v"; grep -h "ssd_step" gpurun_out/pss_$v/run_kernel_stats.csv | cut -c1-150; tail -4 gpurun_out/pss_$v.log
done
unset MSQ_SSD_STEP_ROWS
timeout -k 10 300 python -u -m pytest tests/test_mamba_decode_gpu.py tests/test_generate_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
