#!/bin/bash
# round 2: divided multi-GPU contact search (in-process groups) + C4 per-rank contact cost
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_contact.py tests/test_gpu_decks.py -m gpu > gpurun_out/r2f_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error" gpurun_out/r2f_tests.log | tail -12; tail -3 gpurun_out/r2f_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 4; do
  for d in 1 0; do
    [ $r -eq 1 ] && [ $d -eq 0 ] && continue
    timeout -k 10 300 python -u tools/bench_contact.py --ranks $r --divide $d --steps 40 >> gpurun_out/r2f_contact.jsonl 2>> gpurun_out/r2f_contact.err
    rc=$?; echo "bench ranks=$r divide=$d rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
