#!/bin/bash
# round 3: baseline check of the round-2 code on a fresh box: full GPU suite with durations + smoke + bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=40 tests -m gpu > gpurun_out/r3a_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r3a_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py > gpurun_out/r3a_bench.json 2> gpurun_out/r3a_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r3a_bench.json
exit $rc
