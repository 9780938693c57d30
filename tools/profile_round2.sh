#!/bin/bash
# End-of-round profile (run via gpurun): kernel trace + stats of bench.py (graph replays), then
# one PMC pass per counter group over short eager decodes (FETCH_SIZE and WRITE_SIZE each alone,
# MI355X_MICROARCH.md), summarized on the box (raw CSVs exceed the copy-back limit):
#   gpurun_out/$1.json (tools/profile_summary.py), gpurun_out/$1_kernel_stats.csv, gpurun_out/$1_bench.json
set -e
OUT=$1
R=$GRAFT_REPO_ROOT
D=/tmp/$OUT
mkdir -p $D $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o trace -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c4 > $D/bench_trace.log 2>&1
echo trace done
cp $(find $D -name "trace_kernel_stats.csv" | head -1) $R/gpurun_out/${OUT}_kernel_stats.csv
SHORT="--steps 4 --warmup 1 --no-bs8 --no-c4 --no-cpu-baseline --eager"
run() {  # tag counters extra-args
  timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d $D -o $1 -- python3 $R/bench.py $SHORT $3 > $D/$1.log 2>&1
  echo "$1 rc=$?"
}
run bs1_sqa "SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE" ""
run bs1_sqb "SQ_INSTS_VALU_MFMA_MOPS_BF16,SQ_INSTS_MFMA,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD" ""
run bs1_fetch "FETCH_SIZE" ""
run bs1_write "WRITE_SIZE" ""
find $D -mindepth 2 -name "*.csv" -exec mv {} $D/ \;
python3 $R/tools/profile_summary.py $D $R/gpurun_out/$OUT.json
echo summary done
timeout -k 10 400 python3 $R/bench.py > $R/gpurun_out/${OUT}_bench.json 2> $D/bench.err
echo bench done
