#!/bin/bash
# Round-5 batch P: how much of the batched residual GEMVs is the re-read activation rows: kernel
# traces of bs=8 int4 and C3 with the product and with a timing ablation without the streamed-A
# loads (scratch/noa.so, results wrong by design).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05p
mkdir -p $O
cd $R
export TMPDIR=/tmp
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 0) ;; *) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
for v in base noa; do
  if [ $v = base ]; then L=$R/lit-llama-ja_amd/lit_llama/_lljamd.so; else L=$R/scratch/$v.so; fi
  LLJ_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p8_$v -o run -- \
    python -u bench.py --decode-only --batch 8 --steps 20 > $O/p8_$v.log 2>&1
  chk "trace bs8 $v" $?
  LLJ_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pc3_$v -o run -- \
    python -u bench.py --decode-only --batch 8 --steps 20 --quantize llm.int8 > $O/pc3_$v.log 2>&1
  chk "trace c3 $v" $?
done
exit 0
