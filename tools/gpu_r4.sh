#!/bin/bash
# Round-4 GPU command, one file with named stages (runs on the gpurun box from the repo root):
#   bash tools/gpu_r4.sh STAGE [STAGE ...]
# Every GPU step has its own time limit; the first failing step ends the call (no retries).
# Stages:
#   suite      pytest -m gpu (whole suite, thread timeouts) -> gpurun_out/r4_suite.log
#   smoke      __graft_entry__.smoke()                      -> gpurun_out/r4_smoke.log
#   bench      python bench.py (N = 1, driver defaults)     -> gpurun_out/r4_bench.json
#   rehearse2  python bench.py --gpus 2 with no launcher on the one GPU (ranks share it over RCCL
#              sockets: HAKAI_RCCL_SHARED_GPU=1)           -> gpurun_out/r4_rehearse2.json
#   prof       rocprofv3 kernel trace of a short bench     -> gpurun_out/r4_prof/
#   drift      fused-kernel drift on the reference decks  -> gpurun_out/r4_deck_drift.jsonl
#   c4ranks    C4 contact per rank: one context, 2 and 4 in-process ranks -> gpurun_out/r4_c4_ranks.jsonl
#   c4xslab    the same with C4's elements numbered x slowest (rank ranges = x-slabs) -> gpurun_out/r4_c4_xslab.jsonl
#   c4prof     rocprofv3 kernel trace of the C4 contact run, one context and 2 ranks -> gpurun_out/r4_c4prof_{1,2}$C4TAG/
#              (C4TUNE: extra tuning keys, e.g. contact_filter_memo=0)
#   decks      reference decks end to end, both element modes, graphs -> gpurun_out/r4_decks.jsonl
#   deckprof   rocprofv3 kernel trace of car-crash-N2k, 3200 steps, stream mode -> gpurun_out/r4_deckprof/
#   tests:<pytest -k expr>  a subset of the GPU suite      -> gpurun_out/r4_tests.log
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <seconds> <log> cmd...
    local t=$1 log=$2
    shift 2
    timeout -k 10 "$t" "$@" > "$log" 2>&1
    local rc=$?
    echo "[$(date +%T)] $* -> rc=$rc"
    tail -n 12 "$log"
    return $rc
}
for st in "$@"; do
    case "$st" in
    suite) run 1500 gpurun_out/r4_suite.log python -u -m pytest tests -m gpu -x -v --timeout 300 \
               --timeout-method thread -p no:cacheprovider || exit $? ;;
    smoke) run 300 gpurun_out/r4_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run 600 gpurun_out/r4_bench.json python bench.py || exit $? ;;
    rehearse2) HAKAI_RCCL_SHARED_GPU=1 run 900 gpurun_out/r4_rehearse2.json python bench.py --gpus 2 \
                   --steps 20 --warmup 5 --c5-steps 10 || exit $? ;;
    prof) HAKAI_GRAPH=0 run 600 gpurun_out/r4_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r4_prof \
              -o r4 -- python bench.py --steps 50 --warmup 5 --cpu-baseline 0 || exit $? ;;
    drift) run 600 gpurun_out/r4_deck_drift.jsonl python tools/deck_drift.py || exit $? ;;
    c4ranks) : > gpurun_out/r4_c4_ranks.jsonl
        for r in ${C4RANKS:-1 2 4}; do
            run 600 gpurun_out/r4_c4_ranks_$r.log python tools/bench_contact.py --ranks $r --steps 40 --serial ${C4SERIAL:-1} --tuning "${C4TUNE:-}" || exit $?
            grep '^{' gpurun_out/r4_c4_ranks_$r.log >> gpurun_out/r4_c4_ranks.jsonl
        done ;;
    c4xslab) : > gpurun_out/r4_c4_xslab.jsonl
        for r in 1 2 4; do
            run 600 gpurun_out/r4_c4_xslab_$r.log python tools/bench_contact.py --ranks $r --steps 40 --x-slabs 1 --serial ${C4SERIAL:-1} || exit $?
            grep '^{' gpurun_out/r4_c4_xslab_$r.log >> gpurun_out/r4_c4_xslab.jsonl
        done ;;
    c4prof) for r in ${C4PROF_RANKS:-1 2}; do
            run 600 gpurun_out/r4_c4prof_$r${C4TAG:-}.log rocprofv3 --kernel-trace --stats -d gpurun_out/r4_c4prof_$r${C4TAG:-} -o c4 \
                -- python tools/bench_contact.py --ranks $r --steps 40 --x-slabs ${C4PROF_XSLAB:-0} --tuning "${C4TUNE:-}" || exit $?
        done ;;
    decks) run 900 gpurun_out/r4_decks.jsonl python tools/deck_bench.py --cpu-steps 0 || exit $? ;;
    deckprof) HAKAI_GRAPH=0 run 600 gpurun_out/r4_deckprof.log rocprofv3 --kernel-trace --stats \
                  -d gpurun_out/r4_deckprof -o deck -- python tools/deck_bench.py --decks ${DECK:-car_crash_N2k} \
                  --cpu-steps 0 --modes 1 --max-steps 3200 --tuning graph=0 || exit $? ;;
    tests:*) run 1200 gpurun_out/r4_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 \
                 --timeout-method thread -p no:cacheprovider -k "${st#tests:}" || exit $? ;;
    *) echo "unknown stage $st"; exit 2 ;;
    esac
done
