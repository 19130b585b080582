#!/bin/bash
# round 3: BC application fused into the nodal kernel at any mesh size (fuse_bc 2) against k_bc
# (fuse_bc 1 = only <= 2^18 nodes), with owner-computed assembly, C3 and the C5 slab, both modes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3z
export HAKAI_GRAPH=0
V="bc:fuse_bc=1;fbc:fuse_bc=2;xbc:elem_exact=1,fuse_bc=1;xfbc:elem_exact=1,fuse_bc=2"
for cfg in c3 c5slab; do
  timeout -k 10 300 python -u tools/sweep.py --config $cfg --steps 60 --rounds 4 --variants "$V" > gpurun_out/r3z/sweep_$cfg.log 2>&1
  rc=$?; echo "== $cfg rc=$rc"; cut -c1-140 gpurun_out/r3z/sweep_$cfg.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
