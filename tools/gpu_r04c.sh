#!/bin/bash
# Round-4 batch C: consumer micro-benchmark, engine (K/V prefetch, bigger ring, one-barrier softmax)
# tests + trace, the f16-dequant A/B, the prefill window after the int4 256-row spill fix, engine
# counters, LLM.int8 outlier regimes, the bs=8 FETCH pass that crashed rocprofv3 in rounds 2-3.
# Every GPU step has its own limit; a fault, abort, segfault or time limit ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04c
mkdir -p $O
cd $R
chk() {  # chk <name> <rc>: log; stop on a crash / limit (test failures, rc 1, carry on)
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
for v in 0 1 2 3 4 5 6; do timeout -k 5 30 tools/micro/consume_probe $v 7 2 64 >> $O/consume_probe.log 2>&1; chk "probe $v" $?; done
timeout -k 5 30 tools/micro/consume_probe 0 7 1 64 >> $O/consume_probe.log 2>&1; chk "probe nm1" $?
timeout -k 5 30 tools/micro/consume_probe 0 4 2 64 >> $O/consume_probe.log 2>&1; chk "probe c4" $?
timeout -k 5 30 tools/micro/consume_probe 0 8 2 64 >> $O/consume_probe.log 2>&1; chk "probe c8" $?
timeout -k 10 200 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_engine.log 2>&1
chk "engine tests" $?
if grep -q " passed" $O/t_engine.log && ! grep -q "failed\|error" $O/t_engine.log; then
  timeout -k 10 240 python -u tools/engine_trace.py --out $O/engine_trace.json > $O/engine_trace.log 2>&1; chk trace $?
fi
LLJ_LIB=$R/scratch/eng_f16.so timeout -k 10 200 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_engine_f16.log 2>&1
chk "engine f16 tests" $?
if grep -q " passed" $O/t_engine_f16.log && ! grep -q "failed\|error" $O/t_engine_f16.log; then
  LLJ_LIB=$R/scratch/eng_f16.so timeout -k 10 240 python -u tools/engine_trace.py --out $O/engine_trace_f16.json > $O/engine_trace_f16.log 2>&1
  chk "trace f16" $?
fi
timeout -k 10 200 python -u -m pytest tests/test_generic_gpu.py -k "int8" -q --timeout 120 --timeout-method thread > $O/t_generic_i8.log 2>&1
chk "generic int8" $?
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm or test_attention" -q --timeout 120 --timeout-method thread > $O/t_gemm.log 2>&1
chk "gemm tests" $?
LLJ_GEMM_GLDS=1 timeout -k 10 200 python -u -m pytest tests/test_model_7b_gpu.py -k "prefill" -q --timeout 150 --timeout-method thread > $O/t_prefill.log 2>&1
chk "prefill tests" $?
for cfg in "LLJ_GEMM_GLDS=0" "LLJ_GLDS_COST128=55" "LLJ_GLDS_COST128=0" "LLJ_GLDS_COST128=1000" "LLJ_FLASH_QB=2"; do
  echo "== $cfg" >> $O/prefill_bench.log
  env LLJ_GEMM_GLDS=1 $cfg timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none >> $O/prefill_bench.log 2>&1
  chk "prefill bench $cfg" $?
done
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1); chk list $?
bash tools/engine_pmc.sh r04c_engine_pmc >> $O/status.log 2>&1; chk "engine pmc" $?
for reg in random none 6x20; do
  timeout -k 10 200 python -u tools/i8_outlier_count.py --outliers $reg --batches 8 >> $O/outliers.log 2>&1; chk "outliers $reg" $?
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/bs8f -o bs8_fetch -- python3 $R/bench.py --batch 8 --steps 4 --warmup 1 --no-bs8 --no-c4 --no-cpu-baseline --eager > $O/bs8_fetch.log 2>&1
chk "bs8 fetch" $?
cp -r /tmp/bs8f $O/ 2>/dev/null
exit 0
