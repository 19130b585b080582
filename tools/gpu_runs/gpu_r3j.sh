#!/bin/bash
# round 3: owner pass A/B on ONE box: loop vs branch-free unrolled sums, x keep-t/no-node-prefetch
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HAKAI_GRAPH=0
mkdir -p gpurun_out/r3j
B="-DHK_EXACT_KEEP_T -DHK_EXACT_NO_NODE_PREFETCH"
timeout -k 10 500 tools/variants.sh kn "$B" knu "$B -DHK_OWN_UNROLL" bu "-DHK_OWN_UNROLL" > gpurun_out/r3j/build.log 2>&1
rc=$?; echo "variants build rc=$rc"; [ $rc -eq 0 ] || exit $rc
V="exact_own:elem_exact=1;exact_fe:elem_exact=1,own_assembly=0;fused:elem_exact=0;fused_fe:elem_exact=0,own_assembly=0"
for r in 1 2; do
for lib in base bu kn knu; do
  if [ $lib = base ]; then unset HAKAI_LIB; else export HAKAI_LIB=$PWD/hakai-fem_amd/lib/variants/$lib.so; fi
  timeout -k 10 200 python -u tools/sweep.py --steps 40 --rounds 2 --variants "$V" > gpurun_out/r3j/sweep_${lib}_$r.log 2>&1
  rc=$?; echo "== $lib round $r rc=$rc"; tail -4 gpurun_out/r3j/sweep_${lib}_$r.log; [ $rc -eq 0 ] || exit $rc
done
done
exit 0
