#!/bin/bash
# round 2, final measurements: smoke, C3 bench line, reference decks with the CPU oracle beside them
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2ah_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r2ah_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r2ah_bench.json 2> gpurun_out/r2ah_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/r2ah_bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/deck_bench.py --cpu-steps 2000 > gpurun_out/r2ah_decks.jsonl 2> gpurun_out/r2ah_decks.err
rc=$?; echo "decks rc=$rc"
exit $rc
