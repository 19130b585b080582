#!/bin/bash
# round 3: wave units for owner-computed assembly (one-wave blocks, no block barrier): bit-exact tests,
# then C3 / C5 slab / C4 timing, wave vs block units, both element modes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3q
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_own.py::test_own_wave_units_bitexact > gpurun_out/r3q/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3q/tests.log; [ $rc -eq 0 ] || exit $rc
export HAKAI_GRAPH=0
V="xwave:elem_exact=1,own_unit=2;xblock:elem_exact=1,own_unit=1;fwave:elem_exact=0,own_unit=2;fblock:elem_exact=0,own_unit=1;xfe:elem_exact=1,own_assembly=0;ffe:elem_exact=0,own_assembly=0"
for cfg in c3 c5slab c4; do
  timeout -k 10 300 python -u tools/sweep.py --config $cfg --preload 30 --steps 20 --rounds 2 --variants "$V" > gpurun_out/r3q/sweep_$cfg.log 2>&1
  rc=$?; echo "== $cfg rc=$rc"; cat gpurun_out/r3q/sweep_$cfg.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
done
exit 0
