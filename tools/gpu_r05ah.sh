#!/bin/bash
# Round-5 batch AH: chunk depths of the streamed-workspace int8 GEMVs (AM_I8S), C3 A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ah
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --quantize llm.int8 --variants \
  base dm3:LIB=scratch/dm3.so dm4:LIB=scratch/dm4.so dms3:LIB=scratch/dms3.so > $O/ab_c3.jsonl 2> $O/ab_c3.err
echo "ab c3 rc=$?" >> $O/status.log
exit 0
