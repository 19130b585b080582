#!/bin/bash
# round 3 DIAGNOSTIC (results invalid in the diag variants): where does the reference-order
# element kernel spend its time? exchanges removed / divisions as multiplications / no return
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HAKAI_GRAPH=0
mkdir -p gpurun_out/r3g
B="-DHK_EXACT_KEEP_T -DHK_EXACT_NO_NODE_PREFETCH"
timeout -k 10 500 tools/variants.sh kn "$B" noX "$B -DHK_DIAG_NO_X" noDiv "$B -DHK_DIAG_NO_DIV" noRet "$B -DHK_DIAG_NO_RETURN" all3 "$B -DHK_DIAG_NO_X -DHK_DIAG_NO_DIV -DHK_DIAG_NO_RETURN" > gpurun_out/r3g/build.log 2>&1
rc=$?; echo "variants build rc=$rc"; [ $rc -eq 0 ] || exit $rc
V="exact_fe:elem_exact=1,own_assembly=0;fused_fe:elem_exact=0,own_assembly=0"
for lib in kn noX noDiv noRet all3; do
  export HAKAI_LIB=$PWD/hakai-fem_amd/lib/variants/$lib.so
  timeout -k 10 200 python -u tools/sweep.py --steps 40 --rounds 2 --variants "$V" > gpurun_out/r3g/sweep_$lib.log 2>&1
  rc=$?; echo "== $lib rc=$rc"; tail -2 gpurun_out/r3g/sweep_$lib.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
