#!/bin/bash
# round 3 (final tree): the N>1 bench paths on the one-GPU box -- 2 RCCL ranks under
# torch.distributed.run (sharing the GPU: timings meaningless, the path is what is checked) and
# 8 in-process ranks (HAKAI_RCCL_SHARED_GPU=1: RCCL sees the ranks as separate hosts, socket transport)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3zz
HAKAI_RCCL_SHARED_GPU=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/r3zz/rccl2.json 2> gpurun_out/r3zz/rccl2.err
rc=$?; echo "rccl2 rc=$rc"; cut -c1-600 gpurun_out/r3zz/rccl2.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r3zz/rccl2.err; exit $rc; }
timeout -k 10 400 python -u bench.py --local-ranks 8 --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/r3zz/local8.json 2> gpurun_out/r3zz/local8.err
rc=$?; echo "local8 rc=$rc"; cut -c1-600 gpurun_out/r3zz/local8.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r3zz/local8.err; exit $rc; }
exit 0
