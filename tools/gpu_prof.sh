#!/bin/bash
# Tests + variant sweep + bench + rocprofv3 kernel-trace/stats + PMC (separate passes).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
if [ -n "$SWEEP" ]; then
timeout -k 10 600 python tools/sweep.py --variants "$SWEEP" > gpurun_out/sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep.log | tail -8; ok $rc || exit $rc
fi
timeout -k 10 600 python bench.py --steps 100 --warmup 10 --cpu-seconds 10 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$PROF" ]; then
rm -rf gpurun_out/prof_kt gpurun_out/prof_fetch gpurun_out/prof_write
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --cpu-baseline 0 > gpurun_out/prof_kt.log 2>&1
rc=$?; echo "rocprof kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/prof_fetch.log 2>&1
rc=$?; echo "rocprof fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/prof_write.log 2>&1
rc=$?; echo "rocprof write rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/prof_sq -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/prof_sq.log 2>&1
rc=$?; echo "rocprof sq rc=$rc"
fi
exit 0
