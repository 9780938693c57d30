#!/bin/bash
# round 6 batch C: waves per workgroup of the batched GEMVs (2 waves per SIMD) and bs=8 per-op
# timing ablations (LLJ_ABL 2 no compute / 4 minimal epilogue / 16 no streamed-A loads; wrong outputs)
set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_decode.py --batch 8 --variants base nwm8:LIB=scratch/nwm8.so \
  nws8:LIB=scratch/nws8.so > $O/ab_nw.jsonl 2> $O/ab_nw.err || exit $?
for v in abl2 abl4 abl16; do
  LLJ_LIB=$PWD/scratch/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/p_$v -o run -- python bench.py --decode-only --batch 8 --steps 20 --warmup 5 > $O/p_$v.log 2>&1 || exit $?
  python tools/kstats_db.py /tmp/p_$v > $O/p_$v.csv || exit $?
done
