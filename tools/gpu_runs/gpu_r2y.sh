#!/bin/bash
# round 2: reference-order element mode on C3: persistent pipelined vs one-batch kernel, occupancy variants
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/sweep.py --steps 30 --rounds 4 --variants "fused:;exact:elem_exact=1;exact_batch:elem_exact=1,elem_pipe_blocks=0;exact_batch_w3:elem_exact=1,elem_pipe_blocks=0,elem_minw=3;exact_pipe256:elem_exact=1,elem_pipe_blocks=256" > gpurun_out/r2y_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -6 gpurun_out/r2y_sweep.log
exit $rc
