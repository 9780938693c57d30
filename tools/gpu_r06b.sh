#!/bin/bash
# round 6 batch B: one-read-per-chunk A fragments (LLJ_AFRAG) A/B at bs 1 / 8 and C3, depth / fence
# re-checks on top of it, and the bs=8 decode kernel trace of the new build
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_decode.py --batch 1 8 --variants base afrag0:LIB=scratch/afrag0.so \
  lf1:LIB=scratch/lf1.so dm4:LIB=scratch/dm4.so dms3:LIB=scratch/dms3.so > $O/ab_bs.jsonl 2> $O/ab_bs.err || exit $?
timeout -k 10 300 python -u tools/ab_decode.py --quantize llm.int8 --batch 8 --variants base afrag0:LIB=scratch/afrag0.so \
  > $O/ab_c3.jsonl 2> $O/ab_c3.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8 -o run -- python bench.py --decode-only --batch 8 --steps 20 --warmup 5 > $O/prof8.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run -- python bench.py --decode-only --batch 1 --steps 20 --warmup 5 > $O/prof1.log 2>&1
