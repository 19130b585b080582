#!/bin/bash
# round 3: reference-order kernel variants (keep t in registers / node prefetch), C3, one box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HAKAI_GRAPH=0
mkdir -p gpurun_out/r3f
# build the variants here (keeps the pushed tree small)
timeout -k 10 400 tools/variants.sh keept_nopf "-DHK_EXACT_KEEP_T -DHK_EXACT_NO_NODE_PREFETCH" keept "-DHK_EXACT_KEEP_T" nopf "-DHK_EXACT_NO_NODE_PREFETCH" > gpurun_out/r3f/build.log 2>&1
rc=$?; echo "variants build rc=$rc"; [ $rc -eq 0 ] || exit $rc
V="fused:elem_exact=0;exact_own:elem_exact=1;exact_fe:elem_exact=1,own_assembly=0"
for lib in base keept_nopf keept nopf; do
  if [ $lib = base ]; then unset HAKAI_LIB; else export HAKAI_LIB=$PWD/hakai-fem_amd/lib/variants/$lib.so; fi
  timeout -k 10 200 python -u tools/sweep.py --steps 40 --rounds 3 --variants "$V" > gpurun_out/r3f/sweep_$lib.log 2>&1
  rc=$?; echo "== $lib rc=$rc"; tail -3 gpurun_out/r3f/sweep_$lib.log; [ $rc -eq 0 ] || exit $rc
done
unset HAKAI_LIB
export HAKAI_LIB=$PWD/hakai-fem_amd/lib/variants/keept_nopf.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_exact.py -m gpu > gpurun_out/r3f/exact_keept_nopf.log 2>&1
rc=$?; echo "exact tests keept_nopf rc=$rc"; tail -2 gpurun_out/r3f/exact_keept_nopf.log
exit $rc
