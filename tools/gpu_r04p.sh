#!/bin/bash
# Round-4 batch P: decode attention block size A/B (threads per (row, head) block x keys per
# 16-lane group per pass): product 256 x 8 vs 512 x 4, 512 x 8, 1024 x 2; parity, then decode-only
# tok/s at bs=1 (position ~80: latency-bound, 32 blocks) and bs=8, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04p
mkdir -p $O
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
cd $R
for v in a512 a512u8 a1024; do
  LLJ_LIB=$R/scratch/$v.so timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "attention" -x -q --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1
  chk "tests $v" $?
done
for rep in 1 2; do
  for v in prod a512 a512u8 a1024; do
    if [ $v = prod ]; then unset LLJ_LIB; else export LLJ_LIB=$R/scratch/$v.so; fi
    timeout -k 10 150 python3 bench.py --decode-only --steps 300 --warmup 20 > $O/bs1_${v}_$rep.log 2>&1
    chk "bs1 $v $rep" $?
    timeout -k 10 150 python3 bench.py --decode-only --batch 8 --steps 200 --warmup 20 > $O/bs8_${v}_$rep.log 2>&1
    chk "bs8 $v $rep" $?
  done
done
exit 0
