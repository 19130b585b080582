#!/bin/bash
# round 2: full GPU suite, default bench line, scaling rehearsal lines (local ranks, strong N=1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 900 --timeout-method thread tests -m gpu > gpurun_out/r2c_all.log 2>&1
rc=$?; echo "all rc=$rc"; tail -5 gpurun_out/r2c_all.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r2c_bench.json 2> gpurun_out/r2c_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r2c_bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --local-ranks 8 --steps 50 --warmup 5 > gpurun_out/r2c_local8.json 2> gpurun_out/r2c_local8.err
rc=$?; echo "local8 rc=$rc"; cat gpurun_out/r2c_local8.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --strong --steps 50 --warmup 5 > gpurun_out/r2c_strong1.json 2> gpurun_out/r2c_strong1.err
rc=$?; echo "strong1 rc=$rc"; cat gpurun_out/r2c_strong1.json
exit $rc
