#!/bin/bash
# round 2: mirror fext zero/copy fused into reset/sum, in-process phase B without host round trips:
# multirank + contact + decks suites, then C4 per-rank contact (2 and 4 ranks, drained) and one context
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_contact.py tests/test_gpu_configs.py tests/test_gpu_decks.py -m gpu > gpurun_out/r2x_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r2x_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 4; do
  timeout -k 10 300 python -u tools/bench_contact.py --ranks $r --divide 1 --serial 1 --steps 40 >> gpurun_out/r2x_contact.jsonl 2>> gpurun_out/r2x_contact.err
  rc=$?; echo "bench ranks=$r rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
