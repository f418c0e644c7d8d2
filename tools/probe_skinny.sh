#!/bin/bash
# Per-launch durations of the skinny decode GEMM at probe shapes (overhead structure).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/pprobe -o run --output-format csv -- python -u tools/skinny_bench.py probe > gpurun_out/pprobe.log 2>&1 || exit 1
grep probe gpurun_out/pprobe.log
python - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pprobe/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "skinny" in r["Kernel_Name"]]
d = collections.OrderedDict()
for r in rows:
    k = (r["Kernel_Name"][:60], r.get("Grid_Size_X", r.get("Grid_Size", "?")))
    d.setdefault(k, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in d.items():
    v = sorted(v)
    print(k, len(v), "median us", v[len(v) // 2] / 1e3)
PY
