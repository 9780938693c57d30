#!/bin/bash
# Round-4 batch AC: batched (M <= 8) SwiGLU GEMV chunks in flight per wave, LLJ_DMS 4 (product) vs
# 3 vs 2: parity, then 7B gptq.int4 bs=8 decode-only tok/s interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04ac
mkdir -p $O
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
cd $R
for v in m2 m3; do
  LLJ_LIB=$R/scratch/$v.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "gemv or swiglu" -x -q --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1
  chk "tests $v" $?
done
for rep in 1 2; do
  for v in prod m2 m3; do
    if [ $v = prod ]; then unset LLJ_LIB; else export LLJ_LIB=$R/scratch/$v.so; fi
    timeout -k 10 150 python3 bench.py --decode-only --batch 8 --steps 200 --warmup 20 > $O/bs8_${v}_$rep.log 2>&1
    chk "bs8 $v $rep" $?
  done
done
exit 0
