#!/bin/bash
# r04: the 8-input fold's timing per operand set and its UTCL1 translation counters (tools/fold_tlb_probe.py).
# Each GPU step has its own limit; a time limit or crash ends the call.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
stop() { case $1 in 124|137|134|139) echo "stopping ($1)"; exit "$1" ;; esac; }
timeout -k 10 180 python3 -u tools/fold_tlb_probe.py --first arena > $OUT/fold_tlb_arena_first.jsonl 2> $OUT/fold_tlb_a.err
rc=$?; echo "arena_first rc=$rc"; tail -2 $OUT/fold_tlb_arena_first.jsonl; stop $rc
timeout -k 10 180 python3 -u tools/fold_tlb_probe.py --first separate > $OUT/fold_tlb_separate_first.jsonl 2> $OUT/fold_tlb_s.err
rc=$?; echo "separate_first rc=$rc"; tail -2 $OUT/fold_tlb_separate_first.jsonl; stop $rc
timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum \
    TCP_TCC_READ_REQ_LATENCY_sum --output-format csv -d $OUT/tlb_p1 -o run -- python3 tools/fold_tlb_probe.py --first arena \
    --rounds 1 > $OUT/tlb_p1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"; stop $rc
timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_STALL_MULTI_MISS TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum \
    TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --output-format csv -d $OUT/tlb_p2 -o run \
    -- python3 tools/fold_tlb_probe.py --first arena --rounds 1 > $OUT/tlb_p2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"; stop $rc
echo done
