#!/bin/bash
# Round-4 batch V: bs=1 SwiGLU GEMV chunks in flight per wave (LLJ_D: 4 product, 6, 3; other ops pinned at 4)
# ops, then decode-only tok/s at bs=1 and bs=8, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04v
mkdir -p $O
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
cd $R
for v in sd6 sd3; do
  LLJ_LIB=$R/scratch/$v.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "gemv or swiglu" -x -q --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1
  chk "tests $v" $?
done
for rep in 1 2; do
  for v in prod sd6 sd3; do
    if [ $v = prod ]; then unset LLJ_LIB; else export LLJ_LIB=$R/scratch/$v.so; fi
    timeout -k 10 150 python3 bench.py --decode-only --steps 300 --warmup 20 > $O/bs1_${v}_$rep.log 2>&1
    chk "bs1 $v $rep" $?
    timeout -k 10 150 python3 bench.py --decode-only --batch 8 --steps 200 --warmup 20 > $O/bs8_${v}_$rep.log 2>&1
    chk "bs8 $v $rep" $?
  done
done
exit 0
