#!/bin/bash
# round 3: own_pass without in-pass loads (second-round flag in the prefetched entry); base vs
# keep-t / no-node-prefetch, C3 and the C5 slab
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HAKAI_GRAPH=0
mkdir -p gpurun_out/r3h
timeout -k 10 500 tools/variants.sh keept_nopf "-DHK_EXACT_KEEP_T -DHK_EXACT_NO_NODE_PREFETCH" > gpurun_out/r3h/build.log 2>&1
rc=$?; echo "variants build rc=$rc"; [ $rc -eq 0 ] || exit $rc
V="fused:elem_exact=0;exact_own:elem_exact=1;exact_fe:elem_exact=1,own_assembly=0;fused_fe:own_assembly=0"
for lib in base keept_nopf; do
  if [ $lib = base ]; then unset HAKAI_LIB; else export HAKAI_LIB=$PWD/hakai-fem_amd/lib/variants/$lib.so; fi
  timeout -k 10 200 python -u tools/sweep.py --steps 40 --rounds 3 --variants "$V" > gpurun_out/r3h/sweep_$lib.log 2>&1
  rc=$?; echo "== $lib rc=$rc"; tail -4 gpurun_out/r3h/sweep_$lib.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
