#!/bin/bash
# round 2: the whole GPU suite as the driver runs it at round end, then smoke and the default bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu > gpurun_out/r2ap_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2ap_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2ap_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r2ap_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r2ap_bench.json 2> gpurun_out/r2ap_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r2ap_bench.json
exit $rc
