#!/bin/bash
# round 2, session 2: reference-order (exact) element kernel at 2 vs 3 waves per SIMD on C3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/sweep.py --steps 30 --rounds 3 --variants "exact2:elem_exact=1,elem_minw=2;exact3:elem_exact=1,elem_minw=3;fused:" > gpurun_out/s2p_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/s2p_sweep.log
exit $rc
