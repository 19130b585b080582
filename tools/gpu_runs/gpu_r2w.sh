#!/bin/bash
# round 2: wave-parallel shard prefix + one-scan X1 slots: contact suites, then the C4 contact split
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
true
true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4w_r1 -o c4 -- python3 -u tools/bench_contact.py --ranks 1 --steps 40 > gpurun_out/r2w_r1.log 2>&1
rc=$?; echo "r1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4w_r4 -o c4 -- python3 -u tools/bench_contact.py --ranks 4 --divide 1 --serial 1 --steps 40 > gpurun_out/r2w_r4.log 2>&1
rc=$?; echo "r4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for r in 2 4 4; do
  timeout -k 10 300 python -u tools/bench_contact.py --ranks $r --divide 1 --serial 1 --steps 40 >> gpurun_out/r2w_contact.jsonl 2>> gpurun_out/r2w_contact.err
  rc=$?; echo "bench ranks=$r rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
