#!/bin/bash
# round 6 batch H: L2 prefetch of the weight stream past the register ring (LLJ_PF 3 / 4 / 6 chunks) A/B
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_decode.py --batch 1 8 --variants base pf3:LIB=scratch/pf3.so pf4:LIB=scratch/pf4.so pf6:LIB=scratch/pf6.so > $O/ab.jsonl 2> $O/ab.err
