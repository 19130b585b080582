#!/bin/bash
# round 2, session 2: owner assembly with single-batch passes / finer grids (wide sections): tests,
# then every config with the mode on and off
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_own.py -m gpu > gpurun_out/s2i_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -14 gpurun_out/s2i_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/bench_configs.py > gpurun_out/s2i_configs_own.jsonl 2>gpurun_out/s2i_configs_own.err
rc=$?; echo "configs own rc=$rc"; cat gpurun_out/s2i_configs_own.jsonl; [ $rc -eq 0 ] || exit $rc
HAKAI_OWN_ASSEMBLY=0 timeout -k 10 500 python -u tools/bench_configs.py > gpurun_out/s2i_configs_fe.jsonl 2>gpurun_out/s2i_configs_fe.err
rc=$?; echo "configs fe rc=$rc"; cat gpurun_out/s2i_configs_fe.jsonl
exit $rc
