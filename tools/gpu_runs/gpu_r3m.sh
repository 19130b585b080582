#!/bin/bash
# round 3: banded owner schedule -- owner/exact tests, then C5 slab / C4 / C3 sweeps (contiguous vs banded vs fe)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3m
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_own.py::test_own_banded_two_bodies_contact_bitexact > gpurun_out/r3m/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3m/tests.log; [ $rc -eq 0 ] || exit $rc
V="contig:own_schedule=1;banded:own_schedule=2;fe:own_assembly=0;xcontig:own_schedule=1,elem_exact=1;xbanded:own_schedule=2,elem_exact=1"
for cfg in c5slab c4 c3; do
HAKAI_GRAPH=0 timeout -k 10 300 python -u tools/sweep.py --config $cfg --preload 30 --steps 20 --rounds 2 --variants "$V" > gpurun_out/r3m/sweep_$cfg.log 2>&1
rc=$?; echo "sweep $cfg rc=$rc"; tail -5 gpurun_out/r3m/sweep_$cfg.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
