#!/bin/bash
# round 2: RCCL interface exchange with 2, 3 and 4 ranks sharing the one GPU (socket transport over
# loopback, hakai.dist.rank_device), each bit-exact against one context on the whole bar
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export HAKAI_RCCL_SHARED_GPU=1  # the ranks share the one GPU (hakai.dist.rank_device)
mkdir -p gpurun_out
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
for n in 2 3 4; do
  timeout -k 10 400 $TR --nproc-per-node $n --master-port $((29540 + n)) tools/rccl_exchange_check.py > gpurun_out/r2am_exchange_$n.log 2>&1
  rc=$?; echo "exchange $n rc=$rc"; grep -a "RCCL [0-9]" gpurun_out/r2am_exchange_$n.log | tail -1; [ $rc -eq 0 ] || exit $rc
done
exit 0
