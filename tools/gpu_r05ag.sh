#!/bin/bash
# Round-5 batch AG: bs=8 gptq.int4 A/B: 8-wave attn.c_proj (residual K 4096), residual depth 3.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ag
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --variants \
  base nwr4k:LIB=scratch/nwr4k.so drm3:LIB=scratch/drm3.so > $O/ab_bs8.jsonl 2> $O/ab_bs8.err
echo "ab bs8 rc=$?" >> $O/status.log
exit 0
