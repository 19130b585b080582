#!/bin/bash
# round 3: contact changes -- divided prefilter by 64-id runs, RCCL event all-gather at a grow-only
# capacity (no per-step host sync): multi-rank + RCCL tests, then C4 per-rank contact at 1/2/4 ranks
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3r
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_rccl.py tests/test_gpu_contact.py > gpurun_out/r3r/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3r/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 4; do
  timeout -k 10 300 python -u tools/bench_contact.py --ranks $r --divide 1 --serial 1 --steps 40 >> gpurun_out/r3r/contact.jsonl 2>> gpurun_out/r3r/contact.err
  rc=$?; echo "contact ranks $r rc=$rc"; tail -1 gpurun_out/r3r/contact.jsonl | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
exit 0
