#!/bin/bash
# round 3: lagged barrier-free owner passes with per-wave lists (own_lag): tests, then C3 / C5 slab / C4
# timing of barrier vs lagged passes in both element modes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3w
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_own.py tests/test_gpu_exact.py tests/test_gpu_parity.py > gpurun_out/r3w/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3w/tests.log; [ $rc -eq 0 ] || exit $rc
export HAKAI_GRAPH=0
V="bar:own_lag=0;lag:own_lag=1;xbar:elem_exact=1,own_assembly=2,own_lag=0;xlag:elem_exact=1,own_assembly=2,own_lag=1;xfe:elem_exact=1,own_assembly=0"
for cfg in c3 c5slab c4; do
  timeout -k 10 300 python -u tools/sweep.py --config $cfg --steps 40 --rounds 3 --variants "$V" > gpurun_out/r3w/sweep_$cfg.log 2>&1
  rc=$?; echo "== $cfg rc=$rc"; cut -c1-150 gpurun_out/r3w/sweep_$cfg.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
