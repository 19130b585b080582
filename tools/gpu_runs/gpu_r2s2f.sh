#!/bin/bash
# round 2, session 2: C3 sweep, owner-computed assembly vs fe path (same box, interleaved)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/sweep.py --steps 40 --rounds 4 --variants "base:;own:own_assembly=1;map0:elem_map=0;own_nt0:own_assembly=1,elem_gp_nt=0" > gpurun_out/s2f_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/s2f_sweep.log
exit $rc
