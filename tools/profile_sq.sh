#!/bin/bash
# SQ / GRBM counter passes (MFMA busy, wave waits) over short eager decodes; one pass per
# counter group, each under its own kill timeout. Raw CSVs stay in /tmp/$1 on the box (they
# exceed gpurun's 64 MiB copy-back); the summary lands in gpurun_out/$1.json.
# (llm.int8 bs=8 under --pmc crashed rocprofv3 itself (rc 139): not profiled this way.)
OUT=$1
R=$GRAFT_REPO_ROOT
D=/tmp/$OUT
mkdir -p $D $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
SHORT="--steps 4 --warmup 1 --no-bs8 --no-c4 --no-cpu-baseline --eager"
run() {  # tag counters extra-args
  timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d $D -o $1 -- python3 $R/bench.py $SHORT $3 > $D/$1.log 2>&1
  echo "$1 rc=$?"
}
run bs1_sqa "SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE" ""
run bs1_sqb "SQ_INSTS_VALU_MFMA_MOPS_BF16,SQ_INSTS_MFMA,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD" ""
run c1_sqa "SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE" "--quantize none"
run bs1_fetch "FETCH_SIZE" ""
run bs1_write "WRITE_SIZE" ""
cp $D/*.log $R/gpurun_out/ 2>/dev/null
python3 $R/tools/profile_summary.py $D $R/gpurun_out/$OUT.json
