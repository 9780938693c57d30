#!/bin/bash
# Round-5 batch D: A/B of the new batched-decode defaults (resid depth 4, single-matrix depth 2) against
# further depths, the 256-thread attention, the batch speculative pass; int8 hand-off depth; then the
# PMC repro bisect (stops at the first crash).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05d
mkdir -p $O
cd $R
export TMPDIR=/tmp
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 0) ;; *) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 400 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --variants base drm3:LIB=scratch/drm3.so \
  drm2:LIB=scratch/drm2.so dm3:LIB=scratch/dm3.so att256:LIB=scratch/att256.so specb:SPECB=1 \
  att256specb:LIB=scratch/att256.so,SPECB=1 > $O/ab_bs8.jsonl 2> $O/ab_bs8.err
chk "ab bs8" $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 1 --rounds 3 --steps 60 --variants base att256:LIB=scratch/att256.so \
  > $O/ab_bs1.jsonl 2> $O/ab_bs1.err
chk "ab bs1" $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --quantize llm.int8 --variants base \
  di8q3:LIB=scratch/di8q3.so > $O/ab_c3.jsonl 2> $O/ab_c3.err
chk "ab c3" $?
PMC_CASES="w4:8:4096:4096 i8q:8:4096:4096 i8q:8:4096:11008 i8swiglu:8:11008:4096 i8:8:4096:4096" bash tools/pmc_repro.sh r05d_pmc_repro
echo "pmc repro rc=$?" >> $O/status.log
exit 0
