#!/bin/bash
# round 2: the whole GPU suite on this build, then the C4 contact kernel split
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu > gpurun_out/r2ag_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -cE "PASSED" gpurun_out/r2ag_tests.log; grep -E "FAILED|Error" gpurun_out/r2ag_tests.log | head -5; tail -2 gpurun_out/r2ag_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4ag_r1 -o c4 -- python3 -u tools/bench_contact.py --ranks 1 --steps 40 > gpurun_out/r2ag_r1.log 2>&1
rc=$?; echo "r1 prof rc=$rc"
exit $rc
