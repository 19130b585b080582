#!/bin/bash
# round 2, session 2: full GPU suite, smoke and the default bench line with the final build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/s2j_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/s2j_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2j_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; cat gpurun_out/s2j_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/s2j_bench.json 2> gpurun_out/s2j_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/s2j_bench.json
exit $rc
