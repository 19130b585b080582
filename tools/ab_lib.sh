#!/bin/bash
# A/B of two builds of libhakai_hip.so on the same box: bench.py with the current library, then
# with hakai-fem_amd/lib/libhakai_hip_old.so swapped in, then the current one again.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=hakai-fem_amd/lib
cp $L/libhakai_hip.so /tmp/libhakai_hip_new.so
run() {
  timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --cpu-baseline 0 > gpurun_out/ab_$1.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab_$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['config']['kernel_ms_per_step'])"
}
run new1
cp $L/libhakai_hip_old.so $L/libhakai_hip.so; run old1
cp /tmp/libhakai_hip_new.so $L/libhakai_hip.so; run new2
cp $L/libhakai_hip_old.so $L/libhakai_hip.so; run old2
cp /tmp/libhakai_hip_new.so $L/libhakai_hip.so
