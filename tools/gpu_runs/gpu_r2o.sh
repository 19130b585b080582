#!/bin/bash
# round 2: contact suites after the branch-free pair range; A/B of the round-1 build vs this build on one box (C3 bench)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_contact.py tests/test_gpu_multirank.py tests/test_gpu_configs.py -m gpu > gpurun_out/r2o_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2o_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u abtmp/r1/bench.py --steps 100 --warmup 10 --cpu-baseline 0 > gpurun_out/r2o_ab_r1_$i.json 2>gpurun_out/r2o_ab_r1_$i.err
  rc=$?; echo "r1 bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --cpu-baseline 0 > gpurun_out/r2o_ab_r2_$i.json 2>gpurun_out/r2o_ab_r2_$i.err
  rc=$?; echo "r2 bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
