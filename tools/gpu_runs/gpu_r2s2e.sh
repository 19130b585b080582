#!/bin/bash
# round 2, session 2: fp-contract=on kernels: own vs fe determinism, owner/two-step/parity tests, C3 sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_own2.py > gpurun_out/s2e_diag.log 2>&1
rc=$?; echo "diag rc=$rc"; cat gpurun_out/s2e_diag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_own.py tests/test_gpu_tblock.py tests/test_gpu_parity.py -m gpu > gpurun_out/s2e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -25 gpurun_out/s2e_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/sweep.py --steps 40 --rounds 4 --variants "base:;own:own_assembly=1" > gpurun_out/s2e_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/s2e_sweep.log
exit $rc
