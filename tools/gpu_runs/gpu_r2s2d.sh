#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_own2.py > gpurun_out/s2d_diag.log 2>&1; rc=$?
cat gpurun_out/s2d_diag.log; exit $rc
