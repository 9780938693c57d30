#!/bin/bash
# Round-5 batch I: A/B of the chunk-walk rotation and 8-wave SwiGLU (bs=8 / bs=1 / C3); kernel
# traces of C3 with the prep-kernel timing ablations (scratch/pabl*.so: results wrong by design,
# only the i8_prep_one_kernel durations are read).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05i
mkdir -p $O
cd $R
export TMPDIR=/tmp
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 0) ;; *) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 400 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --variants base rot:LIB=scratch/rot.so \
  nws8:LIB=scratch/nws8.so > $O/ab_bs8.jsonl 2> $O/ab_bs8.err
chk "ab bs8" $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 1 --rounds 3 --steps 60 --variants base rot:LIB=scratch/rot.so \
  > $O/ab_bs1.jsonl 2> $O/ab_bs1.err
chk "ab bs1" $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --quantize llm.int8 --variants base \
  rot:LIB=scratch/rot.so > $O/ab_c3.jsonl 2> $O/ab_c3.err
chk "ab c3" $?
for v in base pabl1 pabl2 pabl4 pabl8 pabl15; do
  if [ $v = base ]; then L=$R/lit-llama-ja_amd/lit_llama/_lljamd.so; else L=$R/scratch/$v.so; fi
  LLJ_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- \
    python -u bench.py --decode-only --batch 8 --steps 20 --quantize llm.int8 > $O/prof_$v.log 2>&1
  chk "trace $v" $?
done
exit 0
