#!/bin/bash
# Round-4 batch C: consumer micro-benchmark, engine (K/V prefetch, bigger ring, one-barrier softmax)
# tests + trace, the f16-dequant A/B, engine counters, LLM.int8 outlier regimes, the bs=8 FETCH pass
# that crashed rocprofv3 in rounds 2-3, the fixed generic int8 test.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04c
mkdir -p $O
cd $R
for v in 0 1 2 3 4; do timeout -k 5 30 tools/micro/consume_probe $v 7 2 64 >> $O/consume_probe.log 2>&1; done
timeout -k 5 30 tools/micro/consume_probe 0 7 1 64 >> $O/consume_probe.log 2>&1
timeout -k 5 30 tools/micro/consume_probe 0 4 2 64 >> $O/consume_probe.log 2>&1
timeout -k 5 30 tools/micro/consume_probe 0 8 2 64 >> $O/consume_probe.log 2>&1
echo "consume probe rc=$?" >> $O/status.log
timeout -k 10 200 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_engine.log 2>&1
echo "engine tests rc=$?" >> $O/status.log
grep -q " passed" $O/t_engine.log && ! grep -q "failed\|error" $O/t_engine.log && \
  timeout -k 10 240 python -u tools/engine_trace.py --out $O/engine_trace.json > $O/engine_trace.log 2>&1
echo "trace rc=$?" >> $O/status.log
LLJ_LIB=$R/scratch/eng_f16.so timeout -k 10 200 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_engine_f16.log 2>&1
echo "engine f16 tests rc=$?" >> $O/status.log
grep -q " passed" $O/t_engine_f16.log && ! grep -q "failed\|error" $O/t_engine_f16.log && \
  LLJ_LIB=$R/scratch/eng_f16.so timeout -k 10 240 python -u tools/engine_trace.py --out $O/engine_trace_f16.json > $O/engine_trace_f16.log 2>&1
echo "trace f16 rc=$?" >> $O/status.log
timeout -k 10 200 python -u -m pytest tests/test_generic_gpu.py -k "int8" -q --timeout 120 --timeout-method thread > $O/t_generic_i8.log 2>&1
echo "generic int8 rc=$?" >> $O/status.log
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1); echo "list rc=$?" >> $O/status.log
bash tools/engine_pmc.sh r04c_engine_pmc >> $O/status.log 2>&1
for reg in random none 6x20; do timeout -k 10 200 python -u tools/i8_outlier_count.py --outliers $reg --batches 8 >> $O/outliers.log 2>&1; done
echo "outlier count rc=$?" >> $O/status.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/bs8f -o bs8_fetch -- python3 $R/bench.py --batch 8 --steps 4 --warmup 1 --no-bs8 --no-c4 --no-cpu-baseline --eager > $O/bs8_fetch.log 2>&1
echo "bs8 fetch rc=$?" >> $O/status.log
