#!/bin/bash
# round 2: triangle search rework (64-B bucket entries with the position, hoisted triangle constants,
# one-wave-per-triangle and prefetch variants): contact + deck suites, then the reference decks and
# C4 contact timed against the previous build (abtmp/base) on the same box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_contact.py tests/test_gpu_decks.py -m gpu > gpurun_out/r2ai_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2ai_tests.log; [ $rc -eq 0 ] || exit $rc
D=car_crash_N2k,car_wall_N2k,Charpy_test,bullet_impact,crash_tube_80_350_solid
for rep in 1 2; do
  timeout -k 10 300 python -u abtmp/base/tools/deck_bench.py --decks $D --modes 1 --cpu-steps 0 --max-steps 40000 >> gpurun_out/r2ai_decks_base.jsonl 2>>gpurun_out/r2ai.err
  rc=$?; echo "base decks rc=$rc"; [ $rc -eq 0 ] || exit $rc
  for t in "" contact_tri_prefetch=1 contact_tri_wave=1 contact_tri_wave=1,contact_tri_prefetch=1; do
    timeout -k 10 300 python -u tools/deck_bench.py --decks $D --modes 1 --cpu-steps 0 --max-steps 40000 --tuning "$t" >> gpurun_out/r2ai_decks_new.jsonl 2>>gpurun_out/r2ai.err
    rc=$?; echo "new decks [$t] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 python -u abtmp/base/tools/bench_contact.py --steps 40 > gpurun_out/r2ai_c4_base.jsonl 2>>gpurun_out/r2ai.err
rc=$?; echo "base c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for t in "" contact_tri_prefetch=1 contact_tri_wave=1 contact_tri_wave=1,contact_tri_prefetch=1; do
  timeout -k 10 300 python -u tools/bench_contact.py --steps 40 --tuning "$t" >> gpurun_out/r2ai_c4_new.jsonl 2>>gpurun_out/r2ai.err
  rc=$?; echo "new c4 [$t] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
