#!/bin/bash
# round 2, session 2: owner passes with a second entry per thread (wide sections at 2 batches per
# pass): owner + multi-rank tests, then every config
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_own.py tests/test_gpu_multirank.py -m gpu > gpurun_out/s2m_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/s2m_tests.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/bench_configs.py > gpurun_out/s2m_configs.jsonl 2>gpurun_out/s2m_configs.err
rc=$?; echo "configs rc=$rc"; cat gpurun_out/s2m_configs.jsonl
exit $rc
