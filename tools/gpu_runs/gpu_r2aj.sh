#!/bin/bash
# round 2: per-kernel times of the reworked triangle search on two self-contact reference decks,
# 32 lanes per triangle (default) vs one wave per triangle (contact_tri_wave=1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export HAKAI_GRAPH=0  # rocprofv3 cannot trace graph launches
mkdir -p gpurun_out
for d in car_wall_N2k crash_tube_80_350_solid car_crash_N2k; do
  for w in 0 1; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_aj_${d}_w$w -o k -- python3 -u tools/deck_bench.py --decks $d --modes 1 --cpu-steps 0 --max-steps 3000 --tuning contact_tri_wave=$w > gpurun_out/r2aj_${d}_w$w.log 2>&1
    rc=$?; echo "$d w=$w rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
