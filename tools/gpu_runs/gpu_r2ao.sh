#!/bin/bash
# round 2: prefilter and binning with unconditional loads (pair box as six 16-B loads): contact, deck and
# contact against the previous build (abtmp/base) on the same box, alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_contact.py tests/test_gpu_decks.py tests/test_gpu_multirank.py tests/test_gpu_configs.py -m gpu > gpurun_out/r2ao_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2ao_tests.log; [ $rc -eq 0 ] || exit $rc
D=car_crash_N2k,car_wall_N2k,Charpy_test,bullet_impact,crash_tube_80_350_solid
for rep in 1 2; do
  timeout -k 10 300 python -u abtmp/base/tools/deck_bench.py --decks $D --modes 1 --cpu-steps 0 >> gpurun_out/r2ao_decks_base.jsonl 2>>gpurun_out/r2ao.err
  rc=$?; echo "base decks rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u tools/deck_bench.py --decks $D --modes 1 --cpu-steps 0 >> gpurun_out/r2ao_decks_new.jsonl 2>>gpurun_out/r2ao.err
  rc=$?; echo "new decks rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u abtmp/base/tools/bench_contact.py --steps 40 >> gpurun_out/r2ao_c4_base.jsonl 2>>gpurun_out/r2ao.err
  rc=$?; echo "base c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u tools/bench_contact.py --steps 40 >> gpurun_out/r2ao_c4_new.jsonl 2>>gpurun_out/r2ao.err
  rc=$?; echo "new c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
