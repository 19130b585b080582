#!/bin/bash
# PMC pass: L2 (TCC) request/hit/miss counts and L1->L2 read requests per kernel of the C3 step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export HAKAI_GRAPH=0  # rocprofv3 cannot trace hipGraph launches
mkdir -p gpurun_out/l2
timeout -s KILL 180 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d gpurun_out/l2/pmc -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/l2/bench.log 2>&1
rc=$?; echo "rocprof l2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/l2/sq -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/l2/bench_sq.log 2>&1
rc=$?; echo "rocprof sq rc=$rc"; exit $rc
