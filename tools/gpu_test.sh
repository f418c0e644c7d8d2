#!/bin/bash
# GPU parity tests only (optionally a subset): tools/gpu_test.sh <tag> [pytest args...]
set -o pipefail
tag=${1:-t}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread "${@:-tests}" > gpurun_out/$tag/pytest.log 2>&1
rc=$?
tail -40 gpurun_out/$tag/pytest.log
exit $rc
