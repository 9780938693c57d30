#!/bin/bash
# Round-4 batch D: the LDS-DMA prefill GEMM after the row-sum fix and the grouped-int4 fix (tests +
# window A/B), two-query-block flash attention, the engine with split MFMA chains, the default bench
# line (in-chain dominant-kernel timing), then the FETCH_SIZE passes over bs=8 and llm.int8 decode
# with the exact dynamic-LDS attribute build (scratch/prof_attr.so; the host SIGSEGV of rounds 2-4).
# Every GPU step has its own limit; a fault, abort, segfault or time limit ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04d
mkdir -p $O
cd $R
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm or attention" -q --timeout 120 --timeout-method thread > $O/t_gemm.log 2>&1
chk "gemm+attention tests" $?
LLJ_GEMM_GLDS=1 timeout -k 10 200 python -u -m pytest tests/test_model_7b_gpu.py -k "prefill" -q --timeout 150 --timeout-method thread > $O/t_prefill.log 2>&1
chk "prefill tests (glds)" $?
for rep in 1 2; do
  for cfg in "LLJ_GEMM_GLDS=0 LLJ_FLASH_QB=1" "LLJ_GEMM_GLDS=1 LLJ_FLASH_QB=1" "LLJ_GEMM_GLDS=1 LLJ_FLASH_QB=2" "LLJ_GEMM_GLDS=0 LLJ_FLASH_QB=2"; do
    echo "== rep $rep $cfg" >> $O/prefill_bench.log
    env $cfg timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 5 >> $O/prefill_bench.log 2>&1
    chk "prefill bench $cfg" $?
  done
done
timeout -k 10 200 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_engine.log 2>&1
chk "engine tests" $?
timeout -k 10 240 python -u tools/engine_trace.py --out $O/engine_trace.json > $O/engine_trace.log 2>&1
chk trace $?
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
chk bench $?
cd /tmp && export TMPDIR=/tmp
LLJ_LIB=$R/scratch/prof_attr.so timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/bs8f -o bs8_fetch -- python3 $R/bench.py --batch 8 --steps 4 --warmup 1 --no-bs8 --no-c4 --no-cpu-baseline --eager > $O/bs8_fetch.log 2>&1
chk "bs8 fetch (exact attr)" $?
cp -r /tmp/bs8f $O/ 2>/dev/null
exit 0
