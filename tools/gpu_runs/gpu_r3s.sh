#!/bin/bash
# round 3: owner slots from the LDS budget (11-bit ids) and band heights at the row optimum:
# owner/exact tests, then C5 slab / C4 sweeps and the one-GPU C5 16 M line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3s
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_own.py tests/test_gpu_exact.py > gpurun_out/r3s/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3s/tests.log; [ $rc -eq 0 ] || exit $rc
export HAKAI_GRAPH=0
V="contig:own_schedule=1;banded:own_schedule=2;fe:own_assembly=0;xauto:elem_exact=1;xown:elem_exact=1,own_assembly=2;xfe:elem_exact=1,own_assembly=0"
for cfg in c5slab c4; do
  timeout -k 10 300 python -u tools/sweep.py --config $cfg --preload 30 --steps 20 --rounds 2 --variants "$V" > gpurun_out/r3s/sweep_$cfg.log 2>&1
  rc=$?; echo "== $cfg rc=$rc"; cat gpurun_out/r3s/sweep_$cfg.log | cut -c1-170; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -u bench.py --strong --steps 30 --warmup 5 --compare-fused 0 > gpurun_out/r3s/strong_n1_c5.json 2> gpurun_out/r3s/strong_n1_c5.err
rc=$?; echo "strong n1 rc=$rc"; tail -1 gpurun_out/r3s/strong_n1_c5.json | cut -c1-1500
exit $rc
