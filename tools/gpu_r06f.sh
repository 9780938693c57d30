#!/bin/bash
# round 6 batch F: attention split into interleaved key ranges, partials merged in attn.c_proj's
# prologue (verdict r5 item 4): parity tests, then the bs=1 A/B against one block per head
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "part_merged or attention" > $O/t.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab_decode.py --batch 1 --rounds 4 --variants base m2:ATT_MERGE=2 m3:ATT_MERGE=3 m4:ATT_MERGE=4 > $O/ab.jsonl 2> $O/ab.err || exit $?
timeout -k 10 200 python -u tools/ab_decode.py --batch 1 --quantize none --rounds 3 --variants base m4:ATT_MERGE=4 > $O/ab_bf16.jsonl 2> $O/ab_bf16.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pc3 -o run -- python bench.py --decode-only --quantize llm.int8 --batch 8 --steps 20 --warmup 5 > $O/pc3.log 2>&1 || exit $?
python tools/kstats_db.py /tmp/pc3 > $O/pc3.csv
timeout -k 10 120 python -u scratch/blas_probe.py > $O/blas.json 2> $O/blas.err
