#!/bin/bash
# Scratch GPU probe of one session step: tools/probe.sh <tag> <cmd...>;
# every step is bounded and the chain stops at the first failure.
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$tag
"$@"
