#!/bin/bash
# round 3: wide-section evidence -- rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE
# passes (separate runs) on C5 16 M (one GPU) and C4; then C4 per-rank contact at 1/2/4 in-process
# ranks and the reference decks end to end
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp HAKAI_GRAPH=0
P=gpurun_out/r3t
rm -rf $P; mkdir -p $P
C5="bench.py --strong --warmup 2 --compare-fused 0 --cpu-baseline 0 --breakdown 0"
C4="tools/bench_contact.py --preload 30"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/c5kt -o run --output-format csv -- python3 $C5 --steps 10 > $P/c5kt.log 2>&1
rc=$?; echo "c5 kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $P/c5f -o run --output-format csv -- python3 $C5 --steps 4 > $P/c5f.log 2>&1
rc=$?; echo "c5 fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $P/c5w -o run --output-format csv -- python3 $C5 --steps 4 > $P/c5w.log 2>&1
rc=$?; echo "c5 write rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/c4kt -o run --output-format csv -- python3 $C4 --steps 20 > $P/c4kt.log 2>&1
rc=$?; echo "c4 kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $P/c4f -o run --output-format csv -- python3 $C4 --steps 5 > $P/c4f.log 2>&1
rc=$?; echo "c4 fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $P/c4w -o run --output-format csv -- python3 $C4 --steps 5 > $P/c4w.log 2>&1
rc=$?; echo "c4 write rc=$rc"; [ $rc -eq 0 ] || exit $rc
for r in 1 2 4; do
  timeout -k 10 300 python -u tools/bench_contact.py --ranks $r --divide 1 --serial 1 --steps 40 >> $P/contact.jsonl 2>> $P/contact.err
  rc=$?; echo "contact ranks $r rc=$rc"; tail -1 $P/contact.jsonl | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
unset HAKAI_GRAPH
timeout -k 10 400 python -u tools/deck_bench.py --cpu-steps 0 > $P/decks.jsonl 2> $P/decks.err
rc=$?; echo "decks rc=$rc"; cut -c1-300 $P/decks.jsonl
exit $rc
