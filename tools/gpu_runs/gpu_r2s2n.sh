#!/bin/bash
# round 2, session 2: final full GPU suite, smoke, C3 bench and the C5 16 M single-GPU (strong) line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/s2n_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/s2n_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2n_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; cat gpurun_out/s2n_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/s2n_bench.json 2> gpurun_out/s2n_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/s2n_bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --strong --steps 30 --warmup 5 --cpu-baseline 0 > gpurun_out/s2n_strong.json 2> gpurun_out/s2n_strong.err
rc=$?; echo "strong rc=$rc"; cat gpurun_out/s2n_strong.json
exit $rc
