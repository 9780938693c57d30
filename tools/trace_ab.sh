#!/bin/bash
# Kernel trace of one decode variant (run via gpurun):
#   tools/trace_ab.sh <name> <batch> [variant spec for tools/ab_decode.py] [quantize mode]
# writes gpurun_out/trace_<name>/{tr_kernel_stats.csv, tail.json (the timed decode steps only)}
set -e
NAME=$1; B=$2; SPEC=${3:-base}; Q=${4:-gptq.int4}
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/trace_$NAME
mkdir -p $D /tmp/tr_$NAME
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tr_$NAME -o tr -- python3 $R/tools/ab_decode.py --variants $SPEC --batch $B --rounds 1 --steps 30 --quantize $Q > $D/ab.log 2>&1
find /tmp/tr_$NAME -name "*kernel_stats.csv" -exec cp {} $D/ \;
python3 $R/tools/trace_tail.py $(find /tmp/tr_$NAME -name "*kernel_trace.csv" | head -1) ${TAIL:-6000} > $D/tail.json
