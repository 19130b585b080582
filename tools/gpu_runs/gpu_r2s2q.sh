#!/bin/bash
# round 2, session 2: owner lists rebuilt on a grid change; owner + multi-rank tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_own.py tests/test_gpu_multirank.py tests/test_gpu_tblock.py -m gpu > gpurun_out/s2q_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/s2q_tests.log | tail -6
exit $rc
