#!/bin/bash
# Round-6 GPU command, one file with named stages (runs on the gpurun box from the repo root):
#   bash tools/gpu_r6.sh STAGE [STAGE ...]
# Every GPU step has its own time limit; the first failing step ends the call (no retries).
# Stages:
#   suite      pytest -m gpu (whole suite, thread timeouts) -> gpurun_out/r6_suite.log
#   smoke      __graft_entry__.smoke()                      -> gpurun_out/r6_smoke.log
#   bench      python bench.py (N = 1, driver defaults)     -> gpurun_out/r6_bench.json
#   prof       rocprofv3 kernel trace of a short bench (MODE=fused|exact) -> gpurun_out/r6_prof_$MODE/
#   sq         rocprofv3 SQ counters of the element kernel (MODE=fused|exact) -> gpurun_out/r6_sq_$MODE/
#   lds        rocprofv3 LDS bank-conflict counters of the element kernel (MODE=fused|exact) -> gpurun_out/r6_lds_$MODE/
#   sweep      tools/sweep.py --variants "$SWEEP" (CONFIG=c3|c4|c5slab) -> gpurun_out/r6_sweep.log
#   diag       per-wave clock totals of the element kernel (variant DIAGLIB, -DHK_DIAG_WAVE) -> gpurun_out/r6_diag_*.jsonl
#   rehearse4  python bench.py --gpus 4 self-launched on the one GPU (RCCL sockets) -> gpurun_out/r6_rehearse4.json
#   rehearse8  the same with --gpus 8 (wall time, per-rank setup and peak RSS in the line) -> gpurun_out/r6_rehearse8.json
#   pmc        calibrated FETCH_SIZE / WRITE_SIZE passes + kernel trace of the C3 bench (MODE=fused|exact)
#              -> gpurun_out/r6_pmc_$MODE/element_pmc.json (profiles/element_pmc{,_exact}.json)
#   window     rocprofv3 kernel trace of the bench's deletion window (C3 steps 7941-7960, both modes)
#              -> gpurun_out/r6_window/ + gpurun_out/r6_window_summary.json (tools/window_trace.py)
#   ablib      LIBS="a b cur" alternating libraries (hakai-fem_amd/lib/variants/<a>.so) under tools/sweep.py
#   contact    tools/bench_contact.py on C4: one context, 2/4 ranks with z- and x-slab ranges -> r6_contact_c4.jsonl
#   envab      ENVV=NAME VALS="0 1": the product library under alternating env values (tools/sweep.py) -> r6_envab.log
#   cgraph     C4 one context without event timers, HAKAI_GRAPH=16 vs 0 alternating -> gpurun_out/r6_cgraph.jsonl
#   pmcwide    FETCH_SIZE / WRITE_SIZE passes + kernel trace on C5 16 M and C4 -> gpurun_out/r6_pmc_{c5,c4}.json
#   tests:<pytest -k expr>  a subset of the GPU suite      -> gpurun_out/r6_tests.log
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
BA="--cpu-baseline 0 --breakdown 0 --deletion-window 0"
for st in "$@"; do
    case "$st" in
    suite) run 1500 gpurun_out/r6_suite.log python -u -m pytest tests -m gpu -x -v --timeout 300 \
               --timeout-method thread -p no:cacheprovider || exit $? ;;
    smoke) run 300 gpurun_out/r6_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run 600 gpurun_out/r6_bench.json python bench.py || exit $? ;;
    prof) M=${MODE:-fused}; P=gpurun_out/r6_prof_$M; rm -rf $P
        HAKAI_GRAPH=0 run 600 gpurun_out/r6_prof_$M.log rocprofv3 --kernel-trace --stats -d $P -o run \
            --output-format csv -- python bench.py --steps 50 --warmup 5 $BA --compare-fused 0 --element-mode $M || exit $? ;;
    sq) M=${MODE:-fused}; P=gpurun_out/r6_sq_$M; rm -rf $P
        HAKAI_GRAPH=0 run 300 gpurun_out/r6_sq_$M.log timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU \
            SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
            -d $P -o run --output-format csv -- python bench.py --steps 10 --warmup 2 $BA --compare-fused 0 \
            --element-mode $M || exit $? ;;
    lds) M=${MODE:-exact}; P=gpurun_out/r6_lds_$M; rm -rf $P
        HAKAI_GRAPH=0 run 300 gpurun_out/r6_lds_$M.log timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT \
            SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES -d $P -o run --output-format csv -- python bench.py --steps 10 \
            --warmup 2 $BA --compare-fused 0 --element-mode $M || exit $? ;;
    sweep) run 900 gpurun_out/r6_sweep.log python tools/sweep.py --config ${CONFIG:-c3} --rounds ${ROUNDS:-5} \
               --variants "$SWEEP" || exit $? ;;
    diag) V=${DIAGLIB:-diagw}; run 600 gpurun_out/r6_diag_$V.jsonl env HAKAI_LIB=hakai-fem_amd/lib/variants/$V.so \
              python tools/diag_wave.py --config ${CONFIG:-c3} --modes ${MODES:-exact,fused} --tuning "${TUNE:-}" || exit $? ;;
    ablib) : > gpurun_out/r6_ablib.log  # LIBS="a b ..." under hakai-fem_amd/lib/variants (cur = the product library)
        for i in 1 2 3; do
            for v in ${LIBS:-base cur}; do
                if [ $v = cur ]; then lib=hakai-fem_amd/lib/libhakai_hip.so; else lib=hakai-fem_amd/lib/variants/$v.so; fi
                echo "== $v $i" >> gpurun_out/r6_ablib.log
                HAKAI_LIB=$lib run 300 gpurun_out/r6_ablib_cur.log python tools/sweep.py --config ${CONFIG:-c3} \
                    --rounds 2 --variants "${SWEEP:-exact:elem_exact=1;fused:elem_exact=0}" || exit $?
                cat gpurun_out/r6_ablib_cur.log >> gpurun_out/r6_ablib.log
            done
        done
        grep -E "^==|element" gpurun_out/r6_ablib.log ;;
    envab) : > gpurun_out/r6_envab.log  # ENVV=NAME VALS="a b": the product library under alternating env values
        for i in 1 2 3; do
            for v in ${VALS:-0 1}; do
                echo "== ${ENVV}=$v $i" >> gpurun_out/r6_envab.log
                env ${ENVV}=$v timeout -k 10 300 python tools/sweep.py --config ${CONFIG:-c3} --rounds 2 \
                    --variants "${SWEEP:-exact:elem_exact=1;fused:elem_exact=0}" > gpurun_out/r6_envab_cur.log 2>&1 || \
                    { tail -n 20 gpurun_out/r6_envab_cur.log; exit 1; }
                cat gpurun_out/r6_envab_cur.log >> gpurun_out/r6_envab.log
            done
        done
        grep -E "^==|element" gpurun_out/r6_envab.log ;;
    contact) : > gpurun_out/r6_contact_c4.jsonl  # C4 contact per rank: one context, 2 and 4 ranks (z- and x-slabs)
        for spec in "1 0" "2 0" "4 0" "2 1" "4 1"; do
            set -- $spec
            run 600 gpurun_out/r6_contact_cur.log python tools/bench_contact.py --ranks $1 --x-slabs $2 \
                --serial 2 --steps 40 || exit $?
            grep '^{' gpurun_out/r6_contact_cur.log >> gpurun_out/r6_contact_c4.jsonl
        done ;;
    cgraph) : > gpurun_out/r6_cgraph.jsonl  # C4 one context, no event timers: steps from 16-step graphs vs stream mode
        for i in 1 2; do
            for g in 16 0; do
                HAKAI_GRAPH=$g run 600 gpurun_out/r6_cgraph_cur.log python tools/bench_contact.py --profile 0 \
                    --steps 64 || exit $?
                grep '^{' gpurun_out/r6_cgraph_cur.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); \
d.pop('contact_stats_last_step',None); d['HAKAI_GRAPH']=$g; print(json.dumps(d))" >> gpurun_out/r6_cgraph.jsonl || exit $?
            done
        done
        cat gpurun_out/r6_cgraph.jsonl ;;
    rehearse4) HAKAI_RCCL_SHARED_GPU=1 run 900 gpurun_out/r6_rehearse4.json python bench.py --gpus 4 \
                   --steps 20 --warmup 5 --c5-steps 10 || exit $? ;;
    rehearse8) t0=$(date +%s.%N)
        HAKAI_RCCL_SHARED_GPU=1 timeout -k 10 1000 python bench.py --gpus 8 --steps 20 --warmup 5 --c5-steps 10 \
            > gpurun_out/r6_rehearse8.json 2> gpurun_out/r6_rehearse8.err
        rc=$?; t1=$(date +%s.%N)
        echo "{\"wall_s\": $(python -c "print(round($t1 - $t0, 1))"), \"rc\": $rc}" > gpurun_out/r6_rehearse8.wall.json
        echo "[$(date +%T)] rehearse8 -> rc=$rc"; tail -n 5 gpurun_out/r6_rehearse8.err
        cat gpurun_out/r6_rehearse8.wall.json; [ $rc -eq 0 ] || exit $rc ;;
    pmc) M=${MODE:-fused}; P=gpurun_out/r6_pmc_$M; rm -rf $P; mkdir -p $P
        B="--cpu-baseline 0 --breakdown 0 --deletion-window 0 --compare-fused 0 --element-mode $M"
        HAKAI_GRAPH=0 run 600 $P/kt.log rocprofv3 --kernel-trace --stats -d $P/kt -o run --output-format csv -- \
            python bench.py --steps 50 --warmup 5 $B || exit $?
        run 300 $P/calib_fetch.log timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $P/calib_fetch -o run \
            --output-format csv -- tools/_build/pmc_calib || exit $?
        run 300 $P/calib_write.log timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $P/calib_write -o run \
            --output-format csv -- tools/_build/pmc_calib || exit $?
        HAKAI_GRAPH=0 run 600 $P/fetch.log timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run \
            --output-format csv -- python bench.py --steps 10 --warmup 2 $B || exit $?
        HAKAI_GRAPH=0 run 600 $P/write.log timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run \
            --output-format csv -- python bench.py --steps 10 --warmup 2 $B || exit $?
        J=$(grep '^{' $P/kt.log | tail -1)
        ALG=$(echo "$J" | python -c "import json,sys;print(json.load(sys.stdin)['roofline']['alg_bytes_per_launch'])")
        ALGO=$(echo "$J" | python -c "import json,sys;print(json.load(sys.stdin)['roofline']['alg_bytes_per_launch_with_assembly_outputs'])")
        NEL=$(echo "$J" | python -c "import json,sys;print(json.load(sys.stdin)['config']['elements'])")
        python tools/pmc_report.py --calib-fetch $P/calib_fetch --calib-write $P/calib_write --fetch $P/fetch \
            --write $P/write --kt $P/kt --pmc-steps 10 --kt-steps 50 --alg-bytes $ALG --alg-bytes-own $ALGO \
            --element-mode $M --elements $NEL --round r06 --out $P/element_pmc.json > $P/report.log 2>&1 || exit $?
        tail -n 12 $P/report.log ;;
    window) P=gpurun_out/r6_window; rm -rf $P
        HAKAI_GRAPH=0 run 900 $P.log rocprofv3 --kernel-trace --stats -d $P -o run --output-format csv -- \
            python bench.py --steps 20 --warmup 2 --cpu-baseline 0 --breakdown 0 --compare-fused 0 \
            --deletion-window 1 || exit $?
        python tools/window_trace.py --kt $P --log $P.log > gpurun_out/r6_window_summary.json || exit $?
        cat gpurun_out/r6_window_summary.json ;;
    winab) : > gpurun_out/r6_winab.jsonl  # LIBS="a cur": bench lines (idle + deletion window, both modes) alternating
        for i in 1 2; do
            for v in ${LIBS:-base cur}; do
                if [ $v = cur ]; then lib=hakai-fem_amd/lib/libhakai_hip.so; else lib=hakai-fem_amd/lib/variants/$v.so; fi
                HAKAI_LIB=$lib run 400 gpurun_out/r6_winab_cur.log python bench.py --steps 100 --warmup 10 \
                    --cpu-baseline 0 --breakdown 0 || exit $?
                python - "$v" "$i" gpurun_out/r6_winab_cur.log >> gpurun_out/r6_winab.jsonl <<'EOP'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
c = d["config"]; o = c.get("other_mode") or {}; w = c.get("deletion_window") or {}
print(json.dumps({"lib": sys.argv[1], "run": int(sys.argv[2]), "fused_element_ms": d["roofline"]["avg_launch_ms"],
                  "fused_ms_per_step": d["ms_per_step"], "exact_element_ms": o.get("element_avg_ms"),
                  "exact_ms_per_step": o.get("ms_per_step"),
                  "window_fused": {k: w.get("fused", {}).get(k) for k in ("ms_per_step", "element_avg_ms", "deletions")},
                  "window_exact": {k: w.get("exact", {}).get(k) for k in ("ms_per_step", "element_avg_ms", "deletions")}}))
EOP
            done
        done
        cat gpurun_out/r6_winab.jsonl ;;
    wcontrol) P=gpurun_out/r6_wcontrol; rm -rf $P  # the window's hand-off sequence in the idle regime (step 441)
        HAKAI_GRAPH=0 run 600 $P.log rocprofv3 --kernel-trace --stats -d $P -o run --output-format csv -- \
            python tools/window_control.py --first ${FIRST:-441} || exit $?
        python tools/window_trace.py --kt $P --first ${FIRST:-441} > gpurun_out/r6_wcontrol_summary.json || exit $?
        cat gpurun_out/r6_wcontrol_summary.json ;;
    pmcwide) for w in c5 c4; do  # HBM bytes per launch on the wide sections: C5 16 M (--strong, N = 1), C4
            if [ $w = c5 ]; then CMD="python bench.py --strong --steps 10 --warmup 2 $BA --compare-fused 0"
            else CMD="python tools/sweep.py --config c4 --rounds 1 --steps 10 --variants fused:elem_exact=0"; fi
            P=gpurun_out/r6_pmc_$w; rm -rf $P
            HAKAI_GRAPH=0 run 600 $P.kt.log rocprofv3 --kernel-trace -d $P/kt -o run --output-format csv -- $CMD || exit $?
            HAKAI_GRAPH=0 run 600 $P.fetch.log timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run \
                --output-format csv -- $CMD || exit $?
            HAKAI_GRAPH=0 run 600 $P.write.log timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run \
                --output-format csv -- $CMD || exit $?
            python tools/pmc_kernels.py --fetch $P/fetch --write $P/write --kt $P/kt --label $w > $P.json || exit $?
        done ;;
    tests:*) run 1200 gpurun_out/r6_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 \
                 --timeout-method thread -p no:cacheprovider -k "${st#tests:}" || exit $? ;;
    *) echo "unknown stage $st"; exit 2 ;;
    esac
done
