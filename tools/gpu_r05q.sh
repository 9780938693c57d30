#!/bin/bash
# Round-5 batch Q: per-workgroup phase traces of the bs=8 gptq.int4 decode GEMVs (trace build).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05q
mkdir -p $O
cd $R/lit-llama-ja_amd
export TMPDIR=/tmp
timeout -k 10 200 python -u ../tools/phase_trace.py --quantize gptq.int4 --batch 8 --lib scratch/trace.so > $O/phase_bs8.log 2>&1
echo "phase bs8 rc=$?" >> $O/status.log
exit 0
