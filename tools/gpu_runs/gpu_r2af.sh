#!/bin/bash
# round 2: 32-B bucket records + hash parameters in the candidate record: contact suites, C4 contact split, decks
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_contact.py tests/test_gpu_multirank.py tests/test_gpu_decks.py tests/test_gpu_configs.py tests/test_gpu_graph.py -m gpu > gpurun_out/r2af_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r2af_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4af_r1 -o c4 -- python3 -u tools/bench_contact.py --ranks 1 --steps 40 > gpurun_out/r2af_r1.log 2>&1
rc=$?; echo "r1 prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for r in 1 2 4; do
  timeout -k 10 300 python -u tools/bench_contact.py --ranks $r --divide 1 --serial 1 --steps 40 >> gpurun_out/r2af_contact.jsonl 2>> gpurun_out/r2af_contact.err
  rc=$?; echo "bench ranks=$r rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u tools/deck_bench.py --cpu-steps 0 --modes 1 > gpurun_out/r2af_decks.jsonl 2>gpurun_out/r2af_decks.err
rc=$?; echo "decks rc=$rc"
exit $rc
