#!/bin/bash
# Round-4 batch N: QKV epilogue ring-wrap without a division on the common path (parity + timing),
# and the bs=8 A-image LDS cap as a run-time A/B (LLJ_GEMV_LDS_A_KB: 96 = default, 0 = all global-A).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04n
mkdir -p $O
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
cd $R
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_7b_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemv or qkv or decode or generate or batch" > $O/tests.log 2>&1
chk tests $?
for rep in 1 2; do
  for kb in 96 0 48; do
    LLJ_GEMV_LDS_A_KB=$kb timeout -k 10 150 python3 bench.py --decode-only --batch 8 --steps 300 --warmup 20 > $O/bs8_kb${kb}_$rep.log 2>&1
    chk "bs8 kb=$kb rep=$rep" $?
  done
done
timeout -k 10 150 python3 bench.py --decode-only --steps 300 --warmup 20 > $O/bs1.log 2>&1
chk bs1 $?
exit 0
