#!/bin/bash
# round 2: SQ counters of the element kernel, fused vs reference-order (HAKAI_ELEM_EXACT=1) on C3:
# instruction mix and VALU activity, to see what bounds the exact kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=gpurun_out/r2aq
mkdir -p $P
for ex in 0 1; do
  export HAKAI_ELEM_EXACT=$ex
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $P/a$ex -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $P/a$ex.log 2>&1
  rc=$?; echo "pass a exact=$ex rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES -d $P/b$ex -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 > $P/b$ex.log 2>&1
  rc=$?; echo "pass b exact=$ex rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
