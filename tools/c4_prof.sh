#!/bin/bash
# GPU tests (all, or $TESTS) then the C4 contact bench under rocprofv3 kernel-trace/stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/c4
export HAKAI_GRAPH=0  # rocprofv3 cannot trace hipGraph launches
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c4/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/c4/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c4/kt -o run --output-format csv -- python tools/bench_contact.py --steps 50 > gpurun_out/c4/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/c4/bench.log; exit $rc
