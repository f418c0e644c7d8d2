#!/bin/bash
# Same-box A/B(/C...) of environment switches: the given GPU tests under the
# LAST setting, then two rounds of bench runs over the settings in order (per-class
# table printed).
# usage: tools/ab_env.sh "<pytest targets or ->" "<env A>" "<env B>" ["<env C>" ...] [-- bench args]
#   e.g. tools/ab_env.sh - "X=0" "X=1" -- --no-extra
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
tests=$1; shift
envs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
[ "$1" = "--" ] && shift
extra=${*:---no-extra}
last=${envs[${#envs[@]}-1]}
if [ "$tests" != "-" ]; then
  env $last timeout -k 10 400 python -u -m pytest $tests -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab/tests.log; [ $rc = 0 ] || exit 1
fi
run() { tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline $extra > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { tail -20 gpurun_out/ab/$tag.err; return 1; }
  python - "$tag" "$*" <<'EOF'
import json, sys
tag = sys.argv[1]
d = json.load(open(f"gpurun_out/ab/{tag}.json"))
c = d.get("classes", {})
top = sorted(c.items(), key=lambda kv: -kv[1]["ms_per_step"])[:9]
if "ms_per_step" in d:
    print(tag, "[" + sys.argv[2] + "]", d["ms_per_step"], d.get("loss_last"), " ".join(f"{k}={v['ms_per_step']}" for k, v in top))
else:
    print(tag, "[" + sys.argv[2] + "]")
for k in ("decode_cached", "mamba_train", "mamba_decode", "decode"):
    if k in d:
        e = d[k]
        print("   ", k, e.get("ms_per_token_step", e.get("ms_per_step")),
              " ".join(f"{n}={v['ms_per_step']}" for n, v in sorted(e.get("classes", {}).items(), key=lambda kv: -kv[1]["ms_per_step"])[:6]))
EOF
}
for round in 1 2; do
  i=0
  for e in "${envs[@]}"; do
    i=$((i + 1))
    run "c${i}_r${round}" $e || exit 1
  done
done
