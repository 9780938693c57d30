#!/bin/bash
# round 6 batch AF: where the prompt QKV GEMM's epilogue time goes -- kernel traces of the 7B int4
# window with the product and the LLJ_QKV_ABL 1 (no RoPE operand loads) / 2 (no stores) builds
set -o pipefail
O=gpurun_out/r06af
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
for v in base qabl1 qabl2; do
  if [ $v = base ]; then unset LLJ_LIB; else export LLJ_LIB=$R/scratch/$v.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/r06af_$v -o pf -- python3 tools/prefill_bench.py --T 2048 --modes gptq.int4 --iters 2 > $O/prof_$v.log 2>&1 || exit $?
  python3 tools/kstats_db.py /tmp/r06af_$v > $O/pf_$v.csv 2>> $O/kstats.log
done
