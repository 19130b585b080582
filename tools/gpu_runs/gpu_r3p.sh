#!/bin/bash
# round 3: barrier-free owner pass (last-arriving wave runs the pass, HK_OWN_LAST) against the
# block-barrier pass, C3 exact/fused, C5 slab, C4; then the owner/exact tests on the variant
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HAKAI_GRAPH=0
mkdir -p gpurun_out/r3p
V="exact:elem_exact=1;fused:elem_exact=0;xfe:elem_exact=1,own_assembly=0;ffe:elem_exact=0,own_assembly=0"
for r in 1 2; do
for lib in base ol nb; do
  if [ $lib = base ]; then unset HAKAI_LIB; else export HAKAI_LIB=$PWD/hakai-fem_amd/lib/variants/$lib.so; fi
  timeout -k 10 200 python -u tools/sweep.py --steps 40 --rounds 2 --variants "$V" > gpurun_out/r3p/sweep_${lib}_$r.log 2>&1
  rc=$?; echo "== $lib round $r rc=$rc"; head -2 gpurun_out/r3p/sweep_${lib}_$r.log | cut -c1-100; [ $rc -eq 0 ] || exit $rc
done
done
V5="exact:elem_exact=1;fused:elem_exact=0;ffe:elem_exact=0,own_assembly=0"
for lib in base ol; do
  if [ $lib = base ]; then unset HAKAI_LIB; else export HAKAI_LIB=$PWD/hakai-fem_amd/lib/variants/$lib.so; fi
  for cfg in c5slab c4; do
  timeout -k 10 300 python -u tools/sweep.py --config $cfg --preload 30 --steps 20 --rounds 2 --variants "$V5" > gpurun_out/r3p/sweep_${cfg}_${lib}.log 2>&1
  rc=$?; echo "== $cfg $lib rc=$rc"; cat gpurun_out/r3p/sweep_${cfg}_${lib}.log | cut -c1-100; [ $rc -eq 0 ] || exit $rc
  done
done
export HAKAI_LIB=$PWD/hakai-fem_amd/lib/variants/ol.so
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_own.py tests/test_gpu_exact.py > gpurun_out/r3p/tests_ol.log 2>&1
rc=$?; echo "tests ol rc=$rc"; tail -2 gpurun_out/r3p/tests_ol.log
exit $rc
