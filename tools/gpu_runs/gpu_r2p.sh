#!/bin/bash
# round 2: element write-back change (atomic-Q diagnostic): parity suites, then C3 timing default / no assembly / atomic Q
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/sweep.py --steps 40 --rounds 5 --variants "default:;noasm:diag_no_assembly=1;atomicq:diag_atomic_q=1" > gpurun_out/r2p_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -5 gpurun_out/r2p_sweep.log
exit $rc
