#!/bin/bash
# round 2, session 2: every single-GPU config with the owner-assembly default; C5 16 M on one GPU
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/bench_configs.py > gpurun_out/s2h_configs.jsonl 2>gpurun_out/s2h_configs.err
rc=$?; echo "configs rc=$rc"; cat gpurun_out/s2h_configs.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --strong --steps 30 --warmup 5 --cpu-baseline 0 > gpurun_out/s2h_strong.json 2>gpurun_out/s2h_strong.err
rc=$?; echo "strong rc=$rc"; tail -1 gpurun_out/s2h_strong.json
exit $rc
