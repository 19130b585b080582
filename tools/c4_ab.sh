cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/c4
for L in 32 1; do
timeout -k 10 300 python tools/bench_contact.py --steps 50 --tri-lanes $L > gpurun_out/c4/ab_$L.log 2>&1 || exit $?
grep '^{' gpurun_out/c4/ab_$L.log
done
