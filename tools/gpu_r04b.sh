#!/bin/bash
# Round-4 batch B: engine v2 parity + stamp trace, the rocprofv3 --pmc probe (dynamic LDS > 64 KiB),
# the LLM.int8 GEMM tests after the outlier-gather capacity change.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04b
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread > $O/t_engine.log 2>&1
echo "engine tests rc=$?" >> $O/status.log
grep -q "passed" $O/t_engine.log && ! grep -q "failed\|error" $O/t_engine.log && \
  timeout -k 10 240 python -u tools/engine_trace.py --out $O/engine_trace.json > $O/engine_trace.log 2>&1
echo "trace rc=$?" >> $O/status.log
P=$R/tools/micro/pmc_lds_probe
for v in "48 0" "96 160"; do
  timeout -k 5 30 $P $v 4 >> $O/probe_plain.log 2>&1; echo "plain $v rc=$?" >> $O/probe_plain.log
done
cd /tmp && export TMPDIR=/tmp
for v in "48 0" "96 96" "96 160"; do
  set -- $v
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pp_$1_$2 -o p -- $P $1 $2 4 > $O/probe_pmc_$1_$2.log 2>&1
  echo "pmc $v rc=$?" >> $O/status.log
done
cd $R
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "i8 or int8" -q --timeout 120 --timeout-method thread > $O/t_i8.log 2>&1
echo "i8 tests rc=$?" >> $O/status.log
timeout -k 10 300 python -u -m pytest tests/test_model_7b_gpu.py -k "int8" -s -q --timeout 200 --timeout-method thread > $O/t_7b_i8.log 2>&1
echo "7b i8 tests rc=$?" >> $O/status.log
timeout -k 10 300 python -u -m pytest tests/test_fp32_gpu.py tests/test_generic_gpu.py -s -q --timeout 200 --timeout-method thread > $O/t_fp32_generic.log 2>&1
echo "fp32/generic tests rc=$?" >> $O/status.log
