#!/bin/bash
# round 3: C3 owner-list stats, new bench.py (exact headline + fused comparison), SQ counters of
# the reference-order element kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HAKAI_GRAPH=0
mkdir -p gpurun_out/r3d
timeout -k 10 120 python -u tools/c3_stats.py c5 > gpurun_out/r3d/stats.jsonl 2>&1
rc=$?; echo "stats rc=$rc"; cat gpurun_out/r3d/stats.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 100 --cpu-seconds 5 > gpurun_out/r3d/bench.json 2> gpurun_out/r3d/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r3d/bench.json; tail -3 gpurun_out/r3d/bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD -d gpurun_out/r3d/sq -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-baseline 0 --breakdown 0 > gpurun_out/r3d/sq_bench.log 2>&1
rc=$?; echo "sq rc=$rc"
exit $rc
