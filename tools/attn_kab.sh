#!/bin/bash
# Same-box A/B of the attention kernels by rocprofv3 kernel averages (dropout
# p = MB_P, default 0.01): A = the in-tree library, B = the given .so; rounds
# A B A B; prints the per-kernel average us of the attention kernels.
# usage: tools/attn_kab.sh <tag> <libB.so>
set -o pipefail
tag=$1; libb=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
run() { v=$1; lib=$2
  if [ -n "$lib" ]; then export MSQ_LIB_PATH=$lib; else unset MSQ_LIB_PATH; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/$v -o run -- python -u tools/attn_abx.py $v /tmp/kab > gpurun_out/$tag/$v.log 2>&1 || { echo "run $v failed"; tail -5 gpurun_out/$tag/$v.log; return 1; }
  python - "$v" "gpurun_out/$tag/$v/run_results.db" <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[2])
out = []
for n, calls, avg in c.execute("select name, total_calls, average from top_kernels"):
    for k in ("kv5", "fwd3", "bwd_dq", "tri2", "pre_vec", "meta5"):
        if k in n:
            out.append(f"{k} {float(avg):.1f}")
print(sys.argv[1], "  ".join(out), flush=True)
PY
}
run A1 "" && run B1 "$libb" && run A2 "" && run B2 "$libb"
