#!/bin/bash
# round 2, session 2: C5 16 M on one GPU, owner assembly vs fe path, alternating on one box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for own in 1 0; do
    HAKAI_OWN_ASSEMBLY=$own timeout -k 10 400 python -u bench.py --strong --steps 30 --warmup 5 --cpu-baseline 0 > gpurun_out/s2o_strong_${own}_$r.json 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || exit $rc
    python -c "import json; d=json.loads(open('gpurun_out/s2o_strong_${own}_$r.json').read().strip().splitlines()[-1]); print('own=$own run $r', d['ms_per_step'], d['config']['kernel_ms_per_step'])"
  done
done
