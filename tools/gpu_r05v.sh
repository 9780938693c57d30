#!/bin/bash
# Round-5 batch V: per-workgroup phase traces of the bs=8 gptq.int4 and llm.int8 decode GEMVs.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05v
mkdir -p $O
cd $R/lit-llama-ja_amd
export TMPDIR=/tmp
timeout -k 10 200 python -u ../tools/phase_trace.py --quantize gptq.int4 --batch 8 --lib scratch/trace.so > $O/phase_bs8.log 2>&1
rc=$?; echo "phase bs8 rc=$rc" >> $O/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u ../tools/phase_trace.py --quantize llm.int8 --batch 8 --lib scratch/trace.so > $O/phase_c3.log 2>&1
echo "phase c3 rc=$?" >> $O/status.log
exit 0
