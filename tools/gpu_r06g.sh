#!/bin/bash
# round 6 batch G: C3 (7B llm.int8 bs=8) per-op timing ablations of the int8 GEMVs (LLJ_ABL 2 no compute,
# 4 minimal epilogue, 16 no streamed-A loads; outputs wrong by design) + the full-depth int8 test's per-row rels
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
export TMPDIR=/tmp
for v in 2 4 16; do
  LLJ_LIB=$PWD/scratch/c3abl$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/p_$v -o run -- python bench.py --decode-only --quantize llm.int8 --batch 8 --steps 20 --warmup 5 > $O/p_$v.log 2>&1 || exit $?
  python tools/kstats_db.py /tmp/p_$v > $O/p_$v.csv || exit $?
done
timeout -k 10 300 python -u -m pytest tests/test_fulldepth_gpu.py -x -s -q --timeout 250 --timeout-method thread -k int8 > $O/fd8.log 2>&1
