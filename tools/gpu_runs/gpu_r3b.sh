#!/bin/bash
# round 3: new reference-order element kernel (one P2 pass, structural zeros dropped, owner assembly)
# -- exact tests first, then the whole GPU suite, then a C3 A/B of fused vs exact
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_exact.py -m gpu > gpurun_out/r3b_exact.log 2>&1
rc=$?; echo "exact tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r3b_exact.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/sweep.py --rounds 3 --variants "fused:elem_exact=0;exact_own:elem_exact=1;exact_fe:elem_exact=1,own_assembly=0;fused_fe:own_assembly=0" > gpurun_out/r3b_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/r3b_sweep.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=30 tests -m gpu > gpurun_out/r3b_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -4 gpurun_out/r3b_tests.log
exit $rc
