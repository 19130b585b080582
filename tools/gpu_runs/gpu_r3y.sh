#!/bin/bash
# round 3: reference-order kernel with LDS-DMA node staging (elem_stg): bit-exact tests, then C3 timing
# of exact without/with staging (owner sums and fe path) against the fused kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3y
timeout -k 5 60 ./tools/_build/dma_probe > gpurun_out/r3y/dma_probe.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_exact.py tests/test_gpu_own.py tests/test_gpu_parity.py > gpurun_out/r3y/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3y/tests.log; [ $rc -eq 0 ] || exit $rc
export HAKAI_GRAPH=0
V="fused:elem_exact=0;x0:elem_exact=1,elem_stg=0;x1:elem_exact=1,elem_stg=1;xfe0:elem_exact=1,own_assembly=0,elem_stg=0;xfe1:elem_exact=1,own_assembly=0,elem_stg=1"
timeout -k 10 300 python -u tools/sweep.py --config c3 --steps 40 --rounds 3 --variants "$V" > gpurun_out/r3y/sweep_c3.log 2>&1
rc=$?; echo "== c3 rc=$rc"; cut -c1-220 gpurun_out/r3y/sweep_c3.log
exit $rc
