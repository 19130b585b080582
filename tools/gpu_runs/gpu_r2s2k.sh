#!/bin/bash
# round 2, session 2: N-rank bench paths with the final build -- an 8-rank in-process group on the
# one GPU, and bench.py --gpus 2 under torch.distributed.run (RCCL, ranks sharing the GPU)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --local-ranks 8 --steps 50 --warmup 5 > gpurun_out/s2k_local8.json 2> gpurun_out/s2k_local8.err
rc=$?; echo "local8 rc=$rc"; tail -1 gpurun_out/s2k_local8.json; [ $rc -eq 0 ] || exit $rc
export HAKAI_RCCL_SHARED_GPU=1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 30 --warmup 5 > gpurun_out/s2k_rccl2.json 2> gpurun_out/s2k_rccl2.err
rc=$?; echo "rccl2 rc=$rc"; grep '^{' gpurun_out/s2k_rccl2.json | tail -1
exit $rc
