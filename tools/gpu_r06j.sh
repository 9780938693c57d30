#!/bin/bash
# round 6 batch J: the rest of batch I -- bs=8 PMC FETCH / WRITE passes (the bs1 SQ pass ran past its
# 150 s limit in batch I and is skipped), prefill windows, and the batched-GEMV wave-count re-check
set -o pipefail
O=gpurun_out/r06j
R=$PWD
mkdir -p $O /tmp/r06j_pmc
export TMPDIR=/tmp
cd /tmp
A="--batch 8 --steps 4 --warmup 1 --decode-only --eager"
for c in fetch:FETCH_SIZE write:WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc ${c#*:} --output-format csv -d /tmp/r06j_pmc -o bs8_${c%%:*} -- python3 $R/bench.py $A > $R/$O/pmc_${c%%:*}.log 2>&1 || exit $?
done
find /tmp/r06j_pmc -mindepth 2 -name "*.csv" -exec mv {} /tmp/r06j_pmc/ \;
python3 $R/tools/profile_summary.py /tmp/r06j_pmc $R/$O/pmc_bs8.json > $R/$O/pmc_summary.log 2>&1
cd $R
timeout -k 10 300 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 3 > $O/prefill.jsonl 2> $O/prefill.err || exit $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 8 --variants base nwm8:LIB=scratch/nwm8.so nws8:LIB=scratch/nws8.so dms3:LIB=scratch/dmsa3.so > $O/ab_nw.jsonl 2> $O/ab_nw.err
