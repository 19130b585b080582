#!/bin/bash
# Graph-mode check: graph tests first, then the whole GPU suite, the small-deck timings and the bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_graph.log 2>&1
rc=$?; echo "graph tests rc=$rc"; tail -8 gpurun_out/pytest_graph.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python tools/bench_small.py --steps 2000 > gpurun_out/small.log 2>&1
rc=$?; echo "small rc=$rc"; grep '^{' gpurun_out/small.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 100 --warmup 10 --cpu-seconds 10 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | cut -c1-420; exit $rc
