#!/bin/bash
# LLM.int8 decode counters (C3's kernels; run via gpurun): one PMC pass per counter group over
# short eager bs=1 decodes of bench.py's 7B llm.int8 model (bs=8 int8 dispatches use > 64 KiB of
# dynamic LDS, where rocprofv3 --pmc segfaults in the launch path: DESIGN.md §8), summarized on
# the box by tools/profile_summary.py (prefix c3) -> gpurun_out/$1.json
set -e
OUT=$1
R=$GRAFT_REPO_ROOT
D=/tmp/$OUT
mkdir -p $D $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
SHORT="--quantize llm.int8 --batch 1 --steps 4 --warmup 1 --no-bs8 --no-c4 --no-cpu-baseline --eager"
run() {  # tag counters
  timeout -s KILL 150 rocprofv3 --pmc $2 --output-format csv -d $D -o $1 -- python3 $R/bench.py $SHORT > $D/$1.log 2>&1
  echo "$1 rc=$?"
}
run c3_sqa "SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE"
run c3_fetch "FETCH_SIZE"
run c3_write "WRITE_SIZE"
find $D -mindepth 2 -name "*.csv" -exec mv {} $D/ \;
python3 $R/tools/profile_summary.py $D $R/gpurun_out/$OUT.json
echo summary done
