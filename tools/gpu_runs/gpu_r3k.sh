#!/bin/bash
# round 3: owner pass A/B: barrier vs last-arriver pass, x keep-t/no-node-prefetch; then the bit-exact tests on kna
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HAKAI_GRAPH=0
mkdir -p gpurun_out/r3k
B="-DHK_EXACT_KEEP_T -DHK_EXACT_NO_NODE_PREFETCH"
timeout -k 10 500 tools/variants.sh kn "$B" kna "$B -DHK_OWN_ARRIVE" ba "-DHK_OWN_ARRIVE" > gpurun_out/r3k/build.log 2>&1
rc=$?; echo "variants build rc=$rc"; [ $rc -eq 0 ] || exit $rc
V="exact_own:elem_exact=1;exact_fe:elem_exact=1,own_assembly=0;fused:elem_exact=0;fused_fe:elem_exact=0,own_assembly=0"
for r in 1 2; do
for lib in base ba kn kna; do
  if [ $lib = base ]; then unset HAKAI_LIB; else export HAKAI_LIB=$PWD/hakai-fem_amd/lib/variants/$lib.so; fi
  timeout -k 10 200 python -u tools/sweep.py --steps 40 --rounds 2 --variants "$V" > gpurun_out/r3k/sweep_${lib}_$r.log 2>&1
  rc=$?; echo "== $lib round $r rc=$rc"; tail -4 gpurun_out/r3k/sweep_${lib}_$r.log; [ $rc -eq 0 ] || exit $rc
done
done
export HAKAI_LIB=$PWD/hakai-fem_amd/lib/variants/kna.so
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_own.py tests/test_gpu_exact.py > gpurun_out/r3k/tests_kna.log 2>&1
rc=$?; echo "tests kna rc=$rc"; tail -3 gpurun_out/r3k/tests_kna.log
exit $rc
