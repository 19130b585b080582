#!/bin/bash
# round 2: elem_exact defaults to the one-batch kernel: exact/parity/decks/fullsize/configs suites + timing
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_exact.py tests/test_gpu_parity.py tests/test_gpu_decks.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py tests/test_gpu_edges.py -m gpu > gpurun_out/r2z_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r2z_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/sweep.py --steps 30 --rounds 4 --variants "fused:;exact:elem_exact=1;exact_pipe:elem_exact=1,elem_exact_pipe=1" > gpurun_out/r2z_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -4 gpurun_out/r2z_sweep.log
exit $rc
