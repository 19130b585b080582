#!/bin/bash
# round 2: BASELINE configurations under GPU checks (C2/C3/C4/C5) + edge cases
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
true
rc=$?; echo "edges rc=$rc"; tail -8 gpurun_out/r2b_edges.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 1000 python -u -m pytest -v -s --timeout 900 --timeout-method thread tests/test_gpu_configs.py -m gpu -k c4 --durations=0 > gpurun_out/r2b_configs.log 2>&1
rc=$?; echo "configs rc=$rc"; tail -40 gpurun_out/r2b_configs.log
exit $rc
