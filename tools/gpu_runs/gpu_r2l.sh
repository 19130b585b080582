#!/bin/bash
# round 2: multi-rank divided window vs the oracle, car decks fused tolerance, contact suites
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_decks.py -m gpu > gpurun_out/r2l_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/r2l_tests.log | tail -14
exit $rc
