#!/bin/bash
# A/B runs of the C4 contact bench with different probe/tuning flags ($VARIANTS: space-separated arg sets, ',' for spaces)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/c4
i=0
for V in ${VARIANTS:-"--steps,50"}; do
  ARGS=$(echo $V | tr ',' ' ')
  timeout -k 10 300 python tools/bench_contact.py --steps 50 $ARGS > gpurun_out/c4/ab_$i.log 2>&1 || exit $?
  echo "$ARGS"; grep '^{' gpurun_out/c4/ab_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['kernel_ms_per_step'], d['contact_stats_last_step']['events'])"
  i=$((i+1))
done
