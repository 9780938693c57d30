#!/bin/bash
# Round-4 batch A: the rocprofv3 --pmc rc 139 probe (dynamic LDS > 64 KiB) and the LLM.int8 GEMM
# tests after the outlier-gather capacity change.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04a
O=$R/gpurun_out/r04a
P=$R/tools/micro/pmc_lds_probe
for v in "48 0" "96 160" "96 96" "160 160"; do
  timeout -k 5 30 $P $v 4 >> $O/probe_plain.log 2>&1; echo "plain $v rc=$?" >> $O/probe_plain.log
done
cd /tmp && export TMPDIR=/tmp
for v in "48 0" "96 96" "96 160" "160 160"; do
  set -- $v
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pp_$1_$2 -o p -- $P $1 $2 4 > $O/probe_pmc_$1_$2.log 2>&1
  echo "pmc $v rc=$?" >> $O/probe_pmc.log
done
cd $R
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_i8" -x -q --timeout 120 --timeout-method thread > $O/t_i8.log 2>&1
echo "tests rc=$?" >> $O/probe_pmc.log
