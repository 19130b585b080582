#!/bin/bash
# round 2: kernel split of the contact step, one context vs a 4-rank divided group
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4_r1 -o c4 -- python3 -u tools/bench_contact.py --ranks 1 --steps 40 > gpurun_out/r2h_r1.log 2>&1
rc=$?; echo "r1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4_r4 -o c4 -- python3 -u tools/bench_contact.py --ranks 4 --divide 1 --serial 1 --steps 40 > gpurun_out/r2h_r4.log 2>&1
rc=$?; echo "r4 rc=$rc"; exit $rc
