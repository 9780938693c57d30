#!/bin/bash
# Round-4 batch J: flash attention with (long, short) query-block pairs per workgroup: tests + A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04j
mkdir -p $O
cd $R
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "attention_prefill" -q --timeout 120 --timeout-method thread > $O/t_flash.log 2>&1
chk "flash tests" $?
for rep in 1 2; do
  for cfg in "LLJ_FLASH_QB=2 LLJ_FLASH_PAIR=0" "LLJ_FLASH_QB=2 LLJ_FLASH_PAIR=1" "LLJ_FLASH_QB=1 LLJ_FLASH_PAIR=1" "LLJ_FLASH_QB=1 LLJ_FLASH_PAIR=0"; do
    echo "== rep $rep $cfg" >> $O/prefill_bench.log
    env $cfg timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes none gptq.int4 --iters 5 >> $O/prefill_bench.log 2>&1
    chk "prefill bench $cfg" $?
  done
done
exit 0
