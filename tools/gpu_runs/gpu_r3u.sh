#!/bin/bash
# round 3: interior nodes updated in the owner pass (own_fuse_nodal): owner/exact/parity/graph tests,
# then C3 / C5 slab / C2 timing with and without
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3u
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_own.py::test_own_interior_node_update_bitexact tests/test_gpu_graph.py tests/test_gpu_parity.py tests/test_gpu_exact.py > gpurun_out/r3u/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3u/tests.log; [ $rc -eq 0 ] || exit $rc
export HAKAI_GRAPH=0
V="fuse:own_fuse_nodal=1;nofuse:own_fuse_nodal=0;fe:own_assembly=0"
for cfg in c3 c5slab; do
  timeout -k 10 300 python -u tools/sweep.py --config $cfg --steps 40 --rounds 3 --variants "$V" > gpurun_out/r3u/sweep_$cfg.log 2>&1
  rc=$?; echo "== $cfg rc=$rc"; cat gpurun_out/r3u/sweep_$cfg.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --cpu-seconds 5 > gpurun_out/r3u/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/r3u/bench.log | cut -c1-900
exit $rc
