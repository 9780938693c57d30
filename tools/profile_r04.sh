#!/bin/bash
# Round-4 counters (run via gpurun). (1) the decode graph alone under --kernel-trace --stats
# (bench.py --decode-only: in-graph kernel times; bench.py reads the committed summary);
# (2) FETCH / WRITE / SQ passes over eager bs=8 gptq.int4 decodes and llm.int8 decodes at bs=1 and
# bs=8, with the profiling build scratch/prof_lds64.so (LLJ_GEMV_LDS_A_MAX 56 KiB: multi-row
# int4 / bf16 GEMVs read A from global instead of a > 64 KiB LDS image) and LLJ_I8_ROWS=4 (int8
# rows in 4-row slices, 44 KiB images): rocprofv3 --pmc ends in a host SIGSEGV inside
# hipLaunchKernel on dispatches with > 64 KiB of dynamic LDS. Summary:
# gpurun_out/$1.json (tools/profile_summary.py), the graph stats in gpurun_out/$1_graph_stats.csv.
OUT=$1
R=$GRAFT_REPO_ROOT
D=/tmp/$OUT
mkdir -p $D $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/g -o graph -- python3 $R/bench.py --decode-only --steps 100 --warmup 10 > $D/graph.log 2>&1
rc=$?; echo "graph trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
find $D/g -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/${OUT}_graph_stats.csv \;
export LLJ_LIB=$R/scratch/prof_lds64.so
run() {  # tag counters bench-args...
  local tag=$1 ctr=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $D -o $tag -- python3 $R/bench.py "$@" > $D/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"
  case $rc in 0) ;; *) cp $D/$tag.log $R/gpurun_out/ 2>/dev/null; exit $rc;; esac
}
B8="--batch 8 --steps 4 --warmup 1 --no-bs8 --no-c4 --no-cpu-baseline --eager"
C3="--quantize llm.int8 --steps 4 --warmup 1 --no-bs8 --no-c4 --no-cpu-baseline --eager"
run bs8_fetch FETCH_SIZE $B8
run bs8_write WRITE_SIZE $B8
run bs8_sqa "SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE" $B8
export LLJ_I8_ROWS=4
run c3_fetch FETCH_SIZE $C3 --batch 1
run c3_write WRITE_SIZE $C3 --batch 1
run c3_sqa "SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE" $C3 --batch 1
run c3b8_fetch FETCH_SIZE $C3 --batch 8
run c3b8_write WRITE_SIZE $C3 --batch 8
find $D -mindepth 2 -name "*counter_collection.csv" -exec mv {} $D/ \;
python3 $R/tools/profile_summary.py $D $R/gpurun_out/$OUT.json
echo summary done
