#!/bin/bash
# round 2: kernel split of the reference decks' steps (stream mode: rocprofv3 cannot trace graph launches)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export HAKAI_GRAPH=0
mkdir -p gpurun_out
for d in car_wall_N2k; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_deck3_$d -o deck -- python3 -u tools/deck_bench.py --decks $d --cpu-steps 0 --modes 1 --max-steps 3000 > gpurun_out/r2s3_$d.log 2>&1
  rc=$?; echo "$d rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
