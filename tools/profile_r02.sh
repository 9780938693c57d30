#!/bin/bash
# Round-2 profile on the GPU box (run via gpurun): kernel trace + stats of the bench, then one
# PMC pass per counter group (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in passes of their
# own, never with tracing), over short decode runs of every per-layer kernel:
#   bs1   7B gptq.int4 batch 1 (the headline)        FETCH, WRITE, SQ (MFMA busy, waits)
#   c3    7B llm.int8 batch 8 (int8 MFMA)              SQ
#   c1    7B bf16 batch 1                              SQ
# (PMC passes run the decode steps eagerly: counter collection over graph replays stalled.)
# Outputs under gpurun_out/$1/; summarize locally: python tools/profile_summary.py gpurun_out/$1 r02
set -e
OUT=$1
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/$OUT
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
SHORT="--steps 4 --warmup 1 --no-bs8 --no-c4 --no-cpu-baseline --eager"
SQ="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU_MFMA_MOPS_BF16,SQ_INSTS_VALU_MFMA_MOPS_I8,GRBM_GUI_ACTIVE"
if [ -z "$SKIP_TRACE" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o trace -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c4 > $D/bench_trace.log 2>&1
echo trace done
fi
timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D -o bs1_fetch -- python3 $R/bench.py $SHORT > $D/bs1_fetch.log 2>&1
echo fetch done
timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D -o bs1_write -- python3 $R/bench.py $SHORT > $D/bs1_write.log 2>&1
echo write done
timeout -s KILL 170 rocprofv3 --pmc $SQ --output-format csv -d $D -o bs1_sq -- python3 $R/bench.py $SHORT > $D/bs1_sq.log 2>&1
echo sq done
timeout -s KILL 170 rocprofv3 --pmc $SQ --output-format csv -d $D -o c3_sq -- python3 $R/bench.py $SHORT --quantize llm.int8 --batch 8 > $D/c3_sq.log 2>&1
echo c3 done
timeout -s KILL 170 rocprofv3 --pmc $SQ --output-format csv -d $D -o c1_sq -- python3 $R/bench.py $SHORT --quantize none > $D/c1_sq.log 2>&1
echo c1 done
