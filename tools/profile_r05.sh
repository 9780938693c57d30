#!/bin/bash
# Round-5 counter passes (run via gpurun): FETCH_SIZE / WRITE_SIZE / SQ passes, each its own
# rocprofv3 --pmc run, over short eager decodes of bench.py's 7B models: gptq.int4 bs=8 ("bs8") and
# llm.int8 bs=8 ("c3"), then tools/profile_summary.py -> gpurun_out/$1.json (per kernel: HBM bytes
# per launch, traffic / algorithmic bytes, MFMA busy). A pass that fails ends the script (summarized first).
OUT=$1
R=$GRAFT_REPO_ROOT
D=/tmp/$OUT
mkdir -p $D $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
PASSES=${PMC_PASSES:-"bs8 c3"}
run() {  # tag counters bench-args
  local filt=""
  [ -n "$PMC_REGEX" ] && filt="--kernel-include-regex $PMC_REGEX"  # counters of the matching kernels only
  timeout -s KILL 150 rocprofv3 --pmc $2 $filt --output-format csv -d $D -o $1 -- python3 $R/bench.py $3 > $D/$1.log 2>&1
  rc=$?
  echo "$1 rc=$rc" | tee -a $R/gpurun_out/${OUT}_status.log
  tail -3 $D/$1.log >> $R/gpurun_out/${OUT}_status.log
  case $rc in 0) ;; *) summarize; exit $rc;; esac  # nothing more on the GPU after a crash / time limit
}
summarize() {
  find $D -mindepth 2 -name "*.csv" -exec mv {} $D/ \;
  python3 $R/tools/profile_summary.py $D $R/gpurun_out/$OUT.json
}
B8="--batch 8 --steps 4 --warmup 1 --decode-only --eager"
C3="--batch 8 --steps 4 --warmup 1 --decode-only --eager --quantize llm.int8"
SQ="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,GRBM_GUI_ACTIVE"
for p in $PASSES; do
  a=$B8; [ $p = c3 ] && a=$C3; [ $p = bs1 ] && a="--batch 1 --steps 4 --warmup 1 --decode-only --eager"
  run ${p}_fetch "FETCH_SIZE" "$a"
  run ${p}_write "WRITE_SIZE" "$a"
  run ${p}_sq "$SQ" "$a"
done
summarize
echo summary done
