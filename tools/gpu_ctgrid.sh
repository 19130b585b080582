#!/bin/bash
# Contact launch-grid change: contact/graph/deck GPU tests, small-deck timings, C4 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python tools/bench_small.py --only contact --graphs 0,16 --steps 2000 > gpurun_out/small.log 2>&1
rc=$?; echo "small rc=$rc"; grep '^{' gpurun_out/small.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_contact.py --steps 50 > gpurun_out/c4.log 2>&1
rc=$?; echo "c4 rc=$rc"; grep '^{' gpurun_out/c4.log | cut -c1-700; exit $rc
