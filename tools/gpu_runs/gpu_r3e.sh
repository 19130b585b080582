#!/bin/bash
# round 3: is the reference-order element kernel bound by HBM or by its own issue/latency? The same
# A/B on a cache-resident bar (100 k hex, ~190 MB: inside the 256 MB Infinity Cache) and on C3.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HAKAI_GRAPH=0
mkdir -p gpurun_out/r3e
V="fused:elem_exact=0;exact_own:elem_exact=1;exact_fe:elem_exact=1,own_assembly=0;fused_fe:own_assembly=0"
timeout -k 10 200 python -u tools/sweep.py --layers 250 --steps 200 --rounds 3 --variants "$V" > gpurun_out/r3e/sweep_small.log 2>&1
rc=$?; echo "small rc=$rc"; tail -4 gpurun_out/r3e/sweep_small.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/sweep.py --layers 1250 --steps 100 --rounds 3 --variants "$V" > gpurun_out/r3e/sweep_mid.log 2>&1
rc=$?; echo "mid rc=$rc"; tail -4 gpurun_out/r3e/sweep_mid.log
exit $rc
