#!/bin/bash
# round 6 batch U: verdict r5 item 4's second part -- where QKV's excess over its pure stream goes at
# bs=1: decode-graph kernel traces of the product and of the LLJ_ABL 1 (no A prologue) / 4 (minimal
# epilogue) int4 GEMV builds (outputs wrong by design, timing only)
set -o pipefail
O=gpurun_out/r06u
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
for v in base abl1 abl4; do
  if [ $v = base ]; then unset LLJ_LIB; else export LLJ_LIB=$R/scratch/$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r06u_$v -o run -- python3 bench.py --decode-only --batch 1 --steps 20 --warmup 5 > $O/prof_$v.log 2>&1 || exit $?
  python3 tools/kstats_db.py /tmp/r06u_$v > $O/bs1_$v.csv 2>> $O/kstats.log
done
