#!/bin/bash
# Kernel durations and inter-kernel gaps of the Mamba cached decode step
# (tools/decode_prof.py mamba under rocprofv3 --kernel-trace): how much of a
# graph replay is kernel time and how much is launch gap.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
kind=${1:-mamba}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/dgap_$kind -o run --output-format csv -- python -u tools/decode_prof.py $kind 50 > gpurun_out/dgap_$kind.log 2>&1 || { tail -20 gpurun_out/dgap_$kind.log; exit 1; }
cat gpurun_out/dgap_$kind.log
python tools/decode_gaps.py gpurun_out/dgap_$kind
