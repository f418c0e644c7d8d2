cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mprof -o run --output-format csv -- python -u bench.py --only mamba --steps 5 --no-cpu-baseline > gpurun_out/mprof.log 2>&1 || { tail -20 gpurun_out/mprof.log; exit 1; }
f=$(ls gpurun_out/mprof/*kernel_stats.csv gpurun_out/mprof/*/*kernel_stats.csv 2>/dev/null | head -1); echo $f
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{int(r["Calls"]):5d} {float(r["AverageNs"])/1e3:9.1f} us {float(r["TotalDurationNs"])/1e6:8.2f} ms  {r["Name"][:90]}')
PY
