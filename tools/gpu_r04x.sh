#!/bin/bash
# Round-4 batch X: bs=1 SwiGLU GEMV chunks in flight per wave, 4 (product) vs 2 vs 1: parity, 7B
# gptq.int4 decode-only tok/s interleaved, the other bs=1 SwiGLU formats for 2 (config suite), and
# the default bench line with 2.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04x
mkdir -p $O
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
cd $R
LLJ_LIB=$R/scratch/sd1.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "gemv or swiglu" -x -q --timeout 120 --timeout-method thread > $O/t_sd1.log 2>&1
chk "tests sd1" $?
for rep in 1 2; do
  for v in prod sd2 sd1; do
    if [ $v = prod ]; then unset LLJ_LIB; else export LLJ_LIB=$R/scratch/$v.so; fi
    timeout -k 10 150 python3 bench.py --decode-only --steps 300 --warmup 20 > $O/bs1_${v}_$rep.log 2>&1
    chk "bs1 $v $rep" $?
  done
done
export LLJ_LIB=$R/scratch/sd2.so
timeout -k 10 400 python -u tools/config_suite.py --only C1,X-gptq.int8,C4 --out $O/configs_sd2.json > $O/configs_sd2.log 2>&1
chk "configs sd2" $?
timeout -k 10 400 python -u bench.py > $O/bench_sd2.log 2>&1
chk "bench sd2" $?
exit 0
