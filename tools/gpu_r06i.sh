#!/bin/bash
# round 6 batch I: final-build measurements -- GPU suite, smoke, the driver's bench command, kernel traces
# of the decode graph (bs 1 / 8, csv stats), PMC passes (bs1 / bs8 eager decodes), prefill windows, and a
# re-check of the batched-GEMV wave counts on top of the flat epilogue
set -o pipefail
O=gpurun_out/r06i
R=$PWD
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
for b in 1 8; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tr$b -o run -- python bench.py --decode-only --batch $b --steps 20 --warmup 5 > $O/tr$b.log 2>&1 || exit $?
  cp $(find /tmp/tr$b -name "run_kernel_stats.csv" | head -1) $O/graph_bs${b}_kernel_stats.csv || exit $?
done
(cd /tmp && PMC_PASSES="bs1 bs8" bash $R/tools/profile_r05.sh r06_pmc > $R/$O/pmc.log 2>&1) || exit $?
timeout -k 10 300 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 3 > $O/prefill.jsonl 2> $O/prefill.err || exit $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 8 --variants base nwm8:LIB=scratch/nwm8.so nws8:LIB=scratch/nws8.so dms3:LIB=scratch/dmsa3.so > $O/ab_nw.jsonl 2> $O/ab_nw.err
