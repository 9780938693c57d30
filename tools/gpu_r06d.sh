#!/bin/bash
# round 6 batch D: the bs=8 epilogue cost split: stores skipped (LLJ_ABL 32, outputs computed) vs the
# whole epilogue skipped (4) vs the product, kernel traces of bs=8 decode
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
export TMPDIR=/tmp
for v in base abl32 abl4; do
  if [ $v = base ]; then L=$PWD/lit-llama-ja_amd/lit_llama/_lljamd.so; else L=$PWD/scratch/$v.so; fi
  LLJ_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/p_$v -o run -- python bench.py --decode-only --batch 8 --steps 20 --warmup 5 > $O/p_$v.log 2>&1 || exit $?
  python tools/kstats_db.py /tmp/p_$v > $O/p_$v.csv || exit $?
done
