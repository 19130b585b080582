#!/bin/bash
# round 2: contact overflow poison flag + the suites it touches
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_contact.py tests/test_gpu_multirank.py tests/test_gpu_graph.py tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu > gpurun_out/r2e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error" gpurun_out/r2e_tests.log | tail -8; tail -3 gpurun_out/r2e_tests.log
exit $rc
