#!/bin/bash
# round 2, session 2: two-step chunked schedule (tblock_mb): bit-exactness tests, then C3 timing sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tblock.py -m gpu > gpurun_out/s2b_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/s2b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/sweep.py --steps 40 --rounds 3 --variants "base:;tb48:tblock_mb=48;tb96:tblock_mb=96;tb160:tblock_mb=160;tb96nt0:tblock_mb=96,elem_gp_nt=0;tb96nt1:tblock_mb=96,elem_gp_nt=1" > gpurun_out/s2b_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/s2b_sweep.log
exit $rc
