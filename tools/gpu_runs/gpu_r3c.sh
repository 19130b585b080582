#!/bin/bash
# round 3: 32-bit SGPR-based addressing in the element kernels, node prefetch back in exact mode:
# exact + own + parity tests, then the C3 A/B of fused vs exact
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_exact.py tests/test_gpu_own.py tests/test_gpu_parity.py -m gpu > gpurun_out/r3c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r3c_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/sweep.py --rounds 3 --variants "fused:elem_exact=0;exact_own:elem_exact=1;exact_fe:elem_exact=1,own_assembly=0;fused_fe:own_assembly=0" > gpurun_out/r3c_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -5 gpurun_out/r3c_sweep.log
exit $rc
