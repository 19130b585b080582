#!/bin/bash
# round 3 (re-entry): full GPU suite + smoke + default bench on the current tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=30 tests -m gpu > gpurun_out/r3x_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r3x_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3x_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r3x_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py > gpurun_out/r3x_bench.json 2> gpurun_out/r3x_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r3x_bench.json
exit $rc
