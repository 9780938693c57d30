#!/bin/bash
# Round-4 batch G: flash attention with two query blocks per wave as the default, the LDS-DMA GEMM
# with both MFMA steps' fragments read ahead (scratch/glds_pre.so), prefill window A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04g
mkdir -p $O
cd $R
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "glds or attention_prefill" -q --timeout 120 --timeout-method thread > $O/t_kern.log 2>&1
chk "glds+flash tests" $?
LLJ_LIB=$R/scratch/glds_pre.so LLJ_GEMM_GLDS=1 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "glds" -q --timeout 120 --timeout-method thread > $O/t_pre.log 2>&1
chk "glds pre tests" $?
for rep in 1 2; do
  for cfg in "X=0" "LLJ_LIB=$R/scratch/glds_pre.so" "LLJ_LIB=$R/scratch/glds_pre.so LLJ_GEMM_GLDS=1" "LLJ_FLASH_QB=1"; do
    echo "== rep $rep $cfg" >> $O/prefill_bench.log
    env $cfg timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 5 >> $O/prefill_bench.log 2>&1
    chk "prefill bench $cfg" $?
  done
done
exit 0
