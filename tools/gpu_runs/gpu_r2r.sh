#!/bin/bash
# round 2: fused small-deck contact phases: contact/deck/graph/multirank suites, then deck timings fused vs not
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_contact.py tests/test_gpu_decks.py tests/test_gpu_graph.py -m gpu > gpurun_out/r2r_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r2r_tests.log; [ $rc -eq 0 ] || exit $rc
for f in 0 1 0 1; do
  timeout -k 10 300 python -u tools/deck_bench.py --cpu-steps 0 --modes 1 --tuning contact_fuse_small=$f >> gpurun_out/r2r_decks.jsonl 2>>gpurun_out/r2r_decks.err
  rc=$?; echo "decks fuse=$f rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
