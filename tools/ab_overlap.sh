#!/bin/bash
# Same-box A/B: weight-gradient GEMMs on the main stream (default) vs a second stream (--overlap).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abo
for r in 1 2 3; do
  for mode in serial overlap; do
    flag=""; [ $mode = overlap ] && flag="--overlap"
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra $flag > gpurun_out/abo/${mode}_$r.json 2> gpurun_out/abo/${mode}_$r.err || { tail -20 gpurun_out/abo/${mode}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/abo/${mode}_$r.json'));print('$mode', d['ms_per_step'])"
  done
done
