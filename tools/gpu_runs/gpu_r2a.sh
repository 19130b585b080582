#!/bin/bash
# round 2: exact-mode parity tests + full GPU suite + exact vs fused element timing on C3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_exact.py tests/test_gpu_decks.py tests/test_gpu_multirank.py -m gpu > gpurun_out/r2a_exact.log 2>&1
rc=$?; echo "exact rc=$rc"; tail -15 gpurun_out/r2a_exact.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/sweep.py --steps 40 --rounds 4 --variants "fused:elem_exact=0;exact:elem_exact=1" > gpurun_out/r2a_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -5 gpurun_out/r2a_sweep.log
[ $rc -eq 0 ] || exit $rc
exit 0
rc=$?; echo "all rc=$rc"; tail -15 gpurun_out/r2a_all.log
exit $rc
