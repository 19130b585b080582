#!/bin/bash
# One GPU call: driver tests (async VTK output == sync) + end-to-end HAKAI(fname) timing per output mode.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "driver" -p no:cacheprovider > gpurun_out/pytest_driver.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_driver.log; [ $rc -eq 0 ] || exit $rc
df -h /tmp | tail -1
timeout -k 10 600 python -u tools/bench_driver.py --nz ${NZ:-250} --steps ${STEPS:-2000} > gpurun_out/bench_driver.log 2>&1
rc=$?; echo "bench_driver rc=$rc"; cat gpurun_out/bench_driver.log; exit $rc
