#!/bin/bash
# rocprofv3 kernel summaries of the two cached decode steps (tools/decode_prof.py).
# Usage: tools/decode_round.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-decode}
mkdir -p gpurun_out/$tag
for k in transformer mamba; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/$k -o run --output-format csv -- python -u tools/decode_prof.py $k 50 > gpurun_out/$tag/$k.log 2>&1 || { echo "$k failed"; tail -20 gpurun_out/$tag/$k.log; exit 1; }
  tail -4 gpurun_out/$tag/$k.log
done
