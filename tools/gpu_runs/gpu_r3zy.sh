#!/bin/bash
# round 3: reference-order kernel tuning on C3 -- nontemporal Gauss-point streams on/off, grid 512 vs 384
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3zy
export HAKAI_GRAPH=0
V="x:elem_exact=1;xnt0:elem_exact=1,elem_gp_nt=0;x384:elem_exact=1,elem_pipe_blocks=384;f:elem_exact=0;fnt0:elem_exact=0,elem_gp_nt=0"
timeout -k 10 300 python -u tools/sweep.py --config c3 --steps 60 --rounds 4 --variants "$V" > gpurun_out/r3zy/sweep_c3.log 2>&1
rc=$?; echo "== c3 rc=$rc"; cut -c1-140 gpurun_out/r3zy/sweep_c3.log
exit $rc
