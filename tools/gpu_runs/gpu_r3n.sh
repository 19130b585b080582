#!/bin/bash
# round 3: N>1 bench paths with BASELINE config 5 -- the one-GPU C5 16 M line (the c5_strong reference),
# an 8-rank in-process group on the one GPU, and bench.py --gpus 2 under torch.distributed.run (RCCL,
# ranks sharing the GPU over sockets: timings of that line mean nothing, the path and its JSON do)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3n
timeout -k 10 600 python -u bench.py --strong --steps 30 --warmup 5 --compare-fused 0 > gpurun_out/r3n/strong_n1_c5.json 2> gpurun_out/r3n/strong_n1_c5.err
rc=$?; echo "strong n1 rc=$rc"; tail -1 gpurun_out/r3n/strong_n1_c5.json; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/r3n/strong_n1_c5.json profiles/r03_bench_strong_n1_c5.json
timeout -k 10 700 python -u bench.py --local-ranks 8 --steps 30 --warmup 5 --c5-steps 20 --compare-fused 0 > gpurun_out/r3n/local8.json 2> gpurun_out/r3n/local8.err
rc=$?; echo "local8 rc=$rc"; tail -1 gpurun_out/r3n/local8.json; [ $rc -eq 0 ] || exit $rc
export HAKAI_RCCL_SHARED_GPU=1
timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 20 --warmup 5 --c5-steps 10 --compare-fused 0 > gpurun_out/r3n/rccl2.json 2> gpurun_out/r3n/rccl2.err
rc=$?; echo "rccl2 rc=$rc"; grep '^{' gpurun_out/r3n/rccl2.json | tail -1
exit $rc
