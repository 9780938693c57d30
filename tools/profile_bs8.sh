#!/bin/bash
# bs=8 decode counters (run via gpurun): one PMC pass per counter group over short eager bs=8
# decodes of bench.py's 7B gptq.int4 model, summarized on the box by tools/profile_summary.py
# (prefix bs8 -> per-kernel time, HBM bytes vs the M = 8 algorithmic bytes, wait / issue mix).
#   gpurun_out/$1.json
set -e
OUT=$1
R=$GRAFT_REPO_ROOT
D=/tmp/$OUT
mkdir -p $D $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
SHORT="--batch 8 --steps 4 --warmup 1 --no-bs8 --no-c4 --no-cpu-baseline --eager"
run() {  # tag counters
  timeout -s KILL 150 rocprofv3 --pmc $2 --output-format csv -d $D -o $1 -- python3 $R/bench.py $SHORT > $D/$1.log 2>&1
  echo "$1 rc=$?"
}
run bs8_sqa "SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE"
run bs8_sqb "SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_INSTS_SALU"
run bs8_fetch "FETCH_SIZE"
run bs8_write "WRITE_SIZE"
find $D -mindepth 2 -name "*.csv" -exec mv {} $D/ \;
python3 $R/tools/profile_summary.py $D $R/gpurun_out/$OUT.json
echo summary done
