#!/bin/bash
# SQ counters for the C4 contact kernels (one --pmc pass; counters per the guide's limits)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/c4pmc
export HAKAI_GRAPH=0  # rocprofv3 cannot trace hipGraph launches
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR -d gpurun_out/c4pmc/sq -o run --output-format csv -- python tools/bench_contact.py --steps 10 --preload 60 > gpurun_out/c4pmc/sq.log 2>&1
echo rc=$?
