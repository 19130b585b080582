#!/bin/bash
# round 2, session 2: owner-computed assembly: bit-exactness tests, then C3 timing sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_own.py -m gpu > gpurun_out/s2c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/s2c_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/sweep.py --steps 40 --rounds 4 --variants "base:;own:own_assembly=1;own_nt0:own_assembly=1,elem_gp_nt=0" > gpurun_out/s2c_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/s2c_sweep.log
exit $rc
