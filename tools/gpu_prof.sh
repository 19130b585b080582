#!/bin/bash
# Tests + variant sweep + bench + rocprofv3 kernel-trace/stats + PMC (separate passes) + PMC calibration.
# Env switches (pass inline in the gpurun command): SWEEP="variants", PROF=1, NOTEST=1.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
fi
export HAKAI_GRAPH=0  # rocprofv3 cannot trace hipGraph launches; the tests keep the default
if [ -n "$SWEEP" ]; then
timeout -k 10 600 python tools/sweep.py --variants "$SWEEP" > gpurun_out/sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -8 gpurun_out/sweep.log; ok $rc || exit $rc
fi
timeout -k 10 600 python bench.py --steps 100 --warmup 10 --cpu-seconds 10 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$PROF" ]; then
P=gpurun_out/prof
rm -rf $P; mkdir -p $P
KT=50; PS=10
BA="--cpu-baseline 0 --breakdown 0 --compare-fused 0 --element-mode ${MODE:-fused}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $P/kt -o run --output-format csv -- python bench.py --steps $KT --warmup 5 $BA > $P/kt_bench.log 2>&1
rc=$?; echo "rocprof kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $P/calib_fetch -o run --output-format csv -- tools/_build/pmc_calib > $P/calib_fetch.log 2>&1
rc=$?; echo "rocprof calib fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $P/calib_write -o run --output-format csv -- tools/_build/pmc_calib > $P/calib_write.log 2>&1
rc=$?; echo "rocprof calib write rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run --output-format csv -- python bench.py --steps $PS --warmup 2 $BA > $P/fetch_bench.log 2>&1
rc=$?; echo "rocprof fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run --output-format csv -- python bench.py --steps $PS --warmup 2 $BA > $P/write_bench.log 2>&1
rc=$?; echo "rocprof write rc=$rc"; [ $rc -eq 0 ] || exit $rc
ALG=$(python -c "import json;print(json.loads([l for l in open('$P/kt_bench.log') if l.startswith('{')][-1])['roofline']['alg_bytes_per_launch'])")
ALGO=$(python -c "import json;print(json.loads([l for l in open('$P/kt_bench.log') if l.startswith('{')][-1])['roofline']['alg_bytes_per_launch_with_assembly_outputs'])")
NEL=$(python -c "import json;print(json.loads([l for l in open('$P/kt_bench.log') if l.startswith('{')][-1])['config']['elements'])")
python tools/pmc_report.py --calib-fetch $P/calib_fetch --calib-write $P/calib_write --fetch $P/fetch --write $P/write \
  --kt $P/kt --pmc-steps $PS --kt-steps $KT --alg-bytes $ALG --alg-bytes-own $ALGO --element-mode ${MODE:-fused} \
  --elements $NEL --out $P/element_pmc.json > $P/pmc_report.log 2>&1
echo "pmc_report rc=$?"; cat $P/pmc_report.log
if [ -n "$SQ" ]; then
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $P/sq -o run --output-format csv -- python bench.py --steps 10 --warmup 2 $BA > $P/sq_bench.log 2>&1
echo "rocprof sq rc=$?"
fi
fi
exit 0
