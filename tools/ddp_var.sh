#!/bin/bash
# DDP same-data gradient difference (world 2 vs single process) under several
# libraries, twice each: run-to-run spread of the fp32-atomics noise.
# usage: tools/ddp_var.sh lib1.so [lib2.so ...]  ("-" = in-tree)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then unset MSQ_LIB_PATH; else export MSQ_LIB_PATH=$lib; fi
    echo "== $lib"
    timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -q -s --timeout 280 -k "same_data and mamba" 2>&1 | grep -E "grad diff|passed|failed"
    rc=$?; [ $rc -gt 1 ] && exit $rc
  done
done
exit 0
