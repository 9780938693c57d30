#!/bin/bash
# Round-5 batch AC: waves per workgroup of the int8 GEMVs (C3 A/B; variants rebuild csrc/gemv_i8.hip
# only): 8-wave attn.c_proj (residual K 4096), 8-wave norm-fed ops.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ac
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --quantize llm.int8 --variants \
  base nwr4k:LIB=scratch/nwr4k.so nwm8:LIB=scratch/nwm8.so > $O/ab_c3.jsonl 2> $O/ab_c3.err
echo "ab c3 rc=$?" >> $O/status.log
exit 0
