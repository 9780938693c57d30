#!/bin/bash
# round 6 batch AE: C3 without the LLM.int8 statistics hand-off (statistics launches + the streamed
# workspace residual GEMVs, AM_I8S) vs the hand-off, interleaved; kernel trace of the no-hand-off form
set -o pipefail
O=gpurun_out/r06ae
mkdir -p $O
timeout -k 10 300 python -u tools/ab_decode.py --quantize llm.int8 --batch 8 --variants base nohand:I8_HANDOFF=0 > $O/ab.jsonl 2> $O/ab.err || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r06ae_prof -o run -- python3 tools/ab_decode.py --quantize llm.int8 --batch 8 --variants nohand:I8_HANDOFF=0 > $O/prof.log 2>&1 || exit $?
python3 tools/kstats_db.py /tmp/r06ae_prof > $O/c3_nohand_kernel_stats.csv 2> $O/kstats.log
