#!/bin/bash
# Same-box A/B of an environment switch: the given GPU tests under the B
# setting, then alternating bench runs A, B, A, B (per-class table printed).
# usage: tools/ab_env.sh "<pytest targets or ->" "<A env, e.g. X=0>" "<B env, e.g. X=1>" [bench args]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
tests=$1; A=$2; B=$3; shift 3
extra=${*:---no-extra}
if [ "$tests" != "-" ]; then
  env $B timeout -k 10 400 python -u -m pytest $tests -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab/tests.log; [ $rc = 0 ] || exit 1
fi
run() { tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline $extra > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { tail -20 gpurun_out/ab/$tag.err; return 1; }
  python - "$tag" <<'EOF'
import json, sys
tag = sys.argv[1]
d = json.load(open(f"gpurun_out/ab/{tag}.json"))
c = d.get("classes", {})
top = sorted(c.items(), key=lambda kv: -kv[1]["ms_per_step"])[:8]
print(tag, d["ms_per_step"], d.get("loss_last"), " ".join(f"{k}={v['ms_per_step']}" for k, v in top))
for k in ("decode_cached", "mamba_train", "mamba_decode", "decode"):
    if k in d:
        e = d[k]
        print("   ", k, e.get("ms_per_token_step", e.get("ms_per_step")),
              " ".join(f"{n}={v['ms_per_step']}" for n, v in sorted(e.get("classes", {}).items(), key=lambda kv: -kv[1]["ms_per_step"])[:6]))
EOF
}
run A1 $A && run B1 $B && run A2 $A && run B2 $B
