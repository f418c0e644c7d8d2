#!/bin/bash
# Same-box A/B of the Mamba train step (bench.py --only mamba) over settings:
# each argument is "<env assignments> [-- bench flags]", e.g. "X=1 -- --serial"
# usage: tools/mamba_ab.sh "<setting A>" "<setting B>" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mab
for round in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    envs=${e%%--*}; flags=""; [[ "$e" == *--* ]] && flags=${e#*--}
    env $envs timeout -k 10 200 python -u bench.py --only mamba --steps 4 --no-cpu-baseline $flags > gpurun_out/mab/c${i}_r${round}.json 2> gpurun_out/mab/c${i}_r${round}.err || { tail -20 gpurun_out/mab/c${i}_r${round}.err; exit 1; }
    python - "gpurun_out/mab/c${i}_r${round}.json" "$e" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["mamba_train"]
print(sys.argv[2], d["ms_per_step"], " ".join(f"{k}={v['ms_per_step']}" for k, v in list(d["classes"].items())[:8]))
PY
  done
done
