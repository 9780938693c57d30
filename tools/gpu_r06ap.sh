#!/bin/bash
# round 6 batch AP: final-build validation (SwiGLU tail split) -- whole GPU suite, smoke, bench line, prefill windows and a
# kernel trace of the int4 / bf16 windows
set -o pipefail
O=gpurun_out/r06ap
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 200 python -u tools/prefill_bench.py --T 512 1024 2048 --modes gptq.int4 none --iters 4 > $O/prefill.jsonl 2> $O/prefill.err || exit $?
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/r06ap_prof -o pf -- python3 $GRAFT_REPO_ROOT/tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/kstats_db.py /tmp/r06ap_prof > $O/prefill_kernel_stats.csv 2> $O/kstats.log
