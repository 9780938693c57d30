#!/bin/bash
# Round-5 batch U: chunk depths of the int8 GEMVs (C3 A/B; variants rebuild only csrc/gemv_i8.hip).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05u
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --quantize llm.int8 --variants \
  base dm3:LIB=scratch/dm3.so dm4:LIB=scratch/dm4.so dms3:LIB=scratch/dms3.so dms4:LIB=scratch/dms4.so \
  di8q3:LIB=scratch/di8q3.so > $O/ab_c3.jsonl 2> $O/ab_c3.err
echo "ab c3 rc=$?" >> $O/status.log
exit 0
