#!/bin/bash
# round 2: BC fusion at any size (tests) + C3 timing: default / k_bc launch / no force assembly (diagnostic upper bound)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_exact.py tests/test_gpu_edges.py tests/test_gpu_decks.py -m gpu > gpurun_out/r2d_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r2d_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/sweep.py --steps 40 --rounds 5 --variants "default:;kbc:fuse_bc=0;noasm:diag_no_assembly=1;exact:elem_exact=1" > gpurun_out/r2d_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -6 gpurun_out/r2d_sweep.log
exit $rc
