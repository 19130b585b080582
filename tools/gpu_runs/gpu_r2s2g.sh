#!/bin/bash
# round 2, session 2: knobs around owner-computed assembly (BC fusion at any size, nodal order/early loads)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/sweep.py --steps 40 --rounds 4 --variants "own:;fbc2:fuse_bc=2;nrev0:nodal_reverse=0;nearly0:nodal_early=0;fe:own_assembly=0" > gpurun_out/s2g_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/s2g_sweep.log
exit $rc
