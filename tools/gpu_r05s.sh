#!/bin/bash
# Round-5 batch S: the LLM.int8 hand-off test on the product (quant8f) and the packed and scalar
# forms of the fast exact quantization (scratch/fast1.so, fast2.so).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05s
mkdir -p $O
cd $R
export TMPDIR=/tmp
for v in product fast1; do
  if [ $v = product ]; then L=$R/lit-llama-ja_amd/lit_llama/_lljamd.so; else L=$R/scratch/$v.so; fi
  LLJ_LIB=$L timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread -k "statistics_handoff" > $O/t_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc" >> $O/status.log
  case $rc in 0|1) ;; *) exit $rc;; esac
done
timeout -k 10 300 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --quantize llm.int8 --variants \
  quant8f fast1:LIB=scratch/fast1.so > $O/ab_c3.jsonl 2> $O/ab_c3.err
rc=$?; echo "ab c3 rc=$rc" >> $O/status.log; [ $rc -eq 0 ] || exit $rc
cd lit-llama-ja_amd
timeout -k 10 200 python -u ../tools/phase_trace.py --quantize gptq.int4 --batch 8 --lib scratch/trace.so > $O/phase_bs8.log 2>&1
echo "phase bs8 rc=$?" >> $O/status.log
exit 0
