#!/bin/bash
# Round-4 batch K: int4 on the LDS-DMA GEMM with 4 waves along N at 256 x 128 tiles (each B fragment
# dequantized by 2 waves): tests + window A/B against the register-staged default.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04k
mkdir -p $O
cd $R
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "glds" -q --timeout 120 --timeout-method thread > $O/t_glds.log 2>&1
chk "glds tests" $?
for rep in 1 2; do
  for cfg in "X=0" "LLJ_GEMM_GLDS=1"; do
    echo "== rep $rep $cfg" >> $O/prefill_bench.log
    env $cfg timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 --iters 5 >> $O/prefill_bench.log 2>&1
    chk "prefill bench $cfg" $?
  done
done
exit 0
