#!/bin/bash
# round 2: reference decks incl. the v0.0.2 car decks (exact bit-exact, fused parity), deck timings vs the CPU oracle
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_decks.py -m gpu > gpurun_out/r2k_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/r2k_tests.log | tail -14
timeout -k 10 900 python -u tools/deck_bench.py > gpurun_out/r2k_decks.jsonl 2> gpurun_out/r2k_decks.err
rc2=$?; echo "deck bench rc=$rc2"; cat gpurun_out/r2k_decks.jsonl
exit $(( rc | rc2 ))
