#!/bin/bash
# round 6 batch E: the flat batched-row epilogue (LLJ_FLAT_EPI): GPU suite, then A/B at bs 1 / 8 / C3 and the
# bs=8 kernel trace of the new build
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 1 8 --variants base flat0:LIB=scratch/flat0.so > $O/ab_bs.jsonl 2> $O/ab_bs.err || exit $?
timeout -k 10 300 python -u tools/ab_decode.py --quantize llm.int8 --batch 8 --variants base flat0:LIB=scratch/flat0.so > $O/ab_c3.jsonl 2> $O/ab_c3.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/p8 -o run -- python bench.py --decode-only --batch 8 --steps 20 --warmup 5 > $O/p8.log 2>&1 || exit $?
python tools/kstats_db.py /tmp/p8 > $O/p8.csv
