#!/bin/bash
# Round-6 record on one box: the GPU suite, smoke(), the default bench line,
# rocprofv3 kernel summaries (one-stream and timed two-stream train step, Mamba
# step), the PMC traffic passes, and the attention kernels' SQ counters.
# usage: tools/r6_final.sh <tag>
set -o pipefail
tag=${1:-r6fin}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$tag/pytest.log; exit 1; }
tail -1 gpurun_out/$tag/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$tag/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/$tag/smoke.log; exit 1; }
tail -1 gpurun_out/$tag/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || { echo "bench failed"; tail -20 gpurun_out/$tag/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/$tag/bench.json').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['value'], d['mamba_train']['ms_per_step'])"
bash tools/prof_r5.sh $tag || exit 1
bash tools/r6_var.sh $tag/sq "flash_fwd3|flash_bwd_dq|flash_bwd_kv5" pmc - || exit 1
echo done
