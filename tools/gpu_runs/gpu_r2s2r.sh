#!/bin/bash
# round 2, session 2: RCCL ranks with owner-computed assembly, bit-exact against one context
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_rccl.py -m gpu > gpurun_out/s2r_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/s2r_tests.log | tail -10
exit $rc
