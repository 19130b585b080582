#!/bin/bash
# round 3: owner-assembly pass with all contributions loaded at once (branch-free sums)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HAKAI_GRAPH=0
mkdir -p gpurun_out/r3i
B="-DHK_EXACT_KEEP_T -DHK_EXACT_NO_NODE_PREFETCH"
timeout -k 10 500 tools/variants.sh kn "$B" > gpurun_out/r3i/build.log 2>&1
rc=$?; echo "variants build rc=$rc"; [ $rc -eq 0 ] || exit $rc
V="exact_own:elem_exact=1;exact_fe:elem_exact=1,own_assembly=0;fused:elem_exact=0"
for run in kn:2 base:2; do
  lib=${run%%:*}; os=${run##*:}
  if [ $lib = base ]; then unset HAKAI_LIB; else export HAKAI_LIB=$PWD/hakai-fem_amd/lib/variants/$lib.so; fi
  export HAKAI_DIAG_OWN_S=$os
  timeout -k 10 200 python -u tools/sweep.py --steps 40 --rounds 3 --variants "$V" > gpurun_out/r3i/sweep_${lib}_$os.log 2>&1
  rc=$?; echo "== $lib S=$os rc=$rc"; tail -3 gpurun_out/r3i/sweep_${lib}_$os.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
