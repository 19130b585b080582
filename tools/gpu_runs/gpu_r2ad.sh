#!/bin/bash
# round 2: fused fill with the bucket-record loads in flight: contact + decks suites, deck timings (twice)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_decks.py -m gpu > gpurun_out/r2ae_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2ae_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1; do
  timeout -k 10 400 python -u tools/deck_bench.py --cpu-steps 0 --modes 1 >> gpurun_out/r2ae_decks.jsonl 2>>gpurun_out/r2ae_decks.err
  rc=$?; echo "decks rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
