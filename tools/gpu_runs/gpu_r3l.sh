#!/bin/bash
# round 3: restored build (keep-t / no node prefetch default): bit-exact tests + one sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3l
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_own.py tests/test_gpu_exact.py tests/test_gpu_parity.py > gpurun_out/r3l/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3l/tests.log; [ $rc -eq 0 ] || exit $rc
V="exact_own:elem_exact=1;exact_fe:elem_exact=1,own_assembly=0;fused:elem_exact=0;fused_fe:elem_exact=0,own_assembly=0"
HAKAI_GRAPH=0 timeout -k 10 200 python -u tools/sweep.py --steps 40 --rounds 3 --variants "$V" > gpurun_out/r3l/sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -4 gpurun_out/r3l/sweep.log
exit $rc
