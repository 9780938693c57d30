#!/bin/bash
# Round-5 batch Z: ballot-driven outlier walk and two-level code select in the streamed int8 GEMV:
# int8 tests, C3 A/B against the previous build (scratch/prev.so), C3 regimes.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05z
mkdir -p $O
cd $R
export TMPDIR=/tmp
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 0) ;; *) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "int8 or i8 or stat" > $O/t_kern.log 2>&1
chk "kernel tests" $?
timeout -k 10 400 python -u -m pytest tests/test_model_7b_gpu.py tests/test_model_gpu.py tests/test_fulldepth_gpu.py -x -q --timeout 250 --timeout-method thread -k "int8" > $O/t_model.log 2>&1
chk "model tests" $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --quantize llm.int8 --variants \
  new prev:LIB=scratch/prev.so > $O/ab_c3.jsonl 2> $O/ab_c3.err
chk "ab c3" $?
timeout -k 10 300 python -u tools/config_suite.py --only C3,C3-o0,C3-o6x20 --steps 50 > $O/configs.log 2>&1
chk "configs" $?
exit 0
