#!/bin/bash
# round 2: RCCL with more than one rank, on the one-GPU box (hakai.dist.rank_device: the ranks share
# device 0 and look like separate hosts to RCCL, which runs its socket transport over loopback):
# the multi-GPU contact path (divided and replicated, all-gathers + interface send/recv) bit-exact
# against one context, the torchrun HAKAI(fname) driver's VTK files against the one-GPU driver's,
# and bench.py's N-rank line at N = 2 and 4 (timings meaningless: one GPU, socket transport)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export HAKAI_RCCL_SHARED_GPU=1  # the ranks share the one GPU (hakai.dist.rank_device)
mkdir -p gpurun_out
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 400 $TR --nproc-per-node 2 --master-port 29534 tools/rccl_contact_check.py > gpurun_out/r2al_rccl_contact.log 2>&1
rc=$?; echo "rccl contact rc=$rc"; grep -a "RCCL" gpurun_out/r2al_rccl_contact.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/driver_torchrun_smoke.py --nproc 2 > gpurun_out/r2al_driver2.log 2>&1
rc=$?; echo "driver 2 rc=$rc"; tail -2 gpurun_out/r2al_driver2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 $TR --nproc-per-node 2 --master-port 29535 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r2al_bench2.json 2> gpurun_out/r2al_bench2.err
rc=$?; echo "bench 2 rc=$rc"; cat gpurun_out/r2al_bench2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 $TR --nproc-per-node 4 --master-port 29536 bench.py --gpus 4 --steps 10 --warmup 3 > gpurun_out/r2al_bench4.json 2> gpurun_out/r2al_bench4.err
rc=$?; echo "bench 4 rc=$rc"; cat gpurun_out/r2al_bench4.json; [ $rc -eq 0 ] || exit $rc
exit 0
