#!/bin/bash
# round 2, session 2: owner-computed assembly on communicator ranks: multi-rank, RCCL and owner tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_own.py tests/test_gpu_rccl.py tests/test_gpu_configs.py -m gpu > gpurun_out/s2l_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/s2l_tests.log | tail -12
exit $rc
