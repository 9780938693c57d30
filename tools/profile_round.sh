#!/bin/bash
# Round profile on the GPU box (run via gpurun): kernel trace + stats, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md HBM section: never combined with tracing) of the
# same bench command, plus the all-config suite. Outputs under gpurun_out/$1/.
#   summarize locally: python tools/pmc_summary.py gpurun_out/$1 <tag>
set -e
OUT=$1
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$OUT
cd /tmp && export TMPDIR=/tmp
CMD="$R/bench.py --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$OUT -o trace -- python3 $CMD > $R/gpurun_out/$OUT/bench_trace.log 2>&1
# PMC passes on the dominant-kernel loop only (counter collection serializes every dispatch;
# the whole bench under it does not finish in minutes)
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/$OUT -o pmc_fetch -- python3 $CMD --only-dominant > $R/gpurun_out/$OUT/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/$OUT -o pmc_write -- python3 $CMD --only-dominant > $R/gpurun_out/$OUT/bench_write.log 2>&1
timeout -k 10 300 python3 $R/bench.py > $R/gpurun_out/$OUT/bench.json 2> $R/gpurun_out/$OUT/bench.err
timeout -k 10 600 python3 $R/tools/config_suite.py --out $R/gpurun_out/$OUT/configs.json > $R/gpurun_out/$OUT/configs.log 2>&1
