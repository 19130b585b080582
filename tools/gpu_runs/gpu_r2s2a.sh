#!/bin/bash
# round 2, session 2: Infinity Cache probe for two-step chunked element passes + a default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 ./tools/_build/mall_probe 2000000 > gpurun_out/s2a_mall.jsonl 2>&1
rc=$?; echo "mall rc=$rc"; cat gpurun_out/s2a_mall.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/s2a_bench.json 2> gpurun_out/s2a_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/s2a_bench.json
exit $rc
