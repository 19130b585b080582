#!/bin/bash
# round 2: C4 per-rank contact cost, ranks drained one at a time (uncontended per-rank timings)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 2 4; do
  for d in 1 0; do
    timeout -k 10 300 python -u tools/bench_contact.py --ranks $r --divide $d --serial 1 --steps 40 >> gpurun_out/r2g_contact.jsonl 2>> gpurun_out/r2g_contact.err
    rc=$?; echo "bench ranks=$r divide=$d rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
