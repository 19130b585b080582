#!/bin/bash
# round 3: reference-order kernel A/B -- node / Gauss-point loads of the next batch issued before the
# summing pass (prebuilt variants, tools/variants.sh) against the base build, alternating twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HAKAI_GRAPH=0
mkdir -p gpurun_out/r3o
V="exact:elem_exact=1;fused:elem_exact=0;xfe:elem_exact=1,own_assembly=0;ffe:elem_exact=0,own_assembly=0"
for r in 1 2; do
for lib in base en eg enp nb np; do
  if [ $lib = base ]; then unset HAKAI_LIB; else export HAKAI_LIB=$PWD/hakai-fem_amd/lib/variants/$lib.so; fi
  timeout -k 10 200 python -u tools/sweep.py --steps 40 --rounds 2 --variants "$V" > gpurun_out/r3o/sweep_${lib}_$r.log 2>&1
  rc=$?; echo "== $lib round $r rc=$rc"; tail -2 gpurun_out/r3o/sweep_${lib}_$r.log; [ $rc -eq 0 ] || exit $rc
done
done
unset HAKAI_LIB
V4="contig:own_schedule=1;banded:own_schedule=2;fe:own_assembly=0"
timeout -k 10 300 python -u tools/sweep.py --config c4 --preload 30 --steps 20 --rounds 2 --variants "$V4" > gpurun_out/r3o/sweep_c4.log 2>&1
rc=$?; echo "sweep c4 rc=$rc"; tail -3 gpurun_out/r3o/sweep_c4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_exact.py > gpurun_out/r3o/tests_base.log 2>&1
rc=$?; echo "tests base rc=$rc"; tail -2 gpurun_out/r3o/tests_base.log
exit $rc
