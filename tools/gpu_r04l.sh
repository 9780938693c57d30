#!/bin/bash
# Round-4 batch L: int4 LDS-DMA GEMM with 4 waves along N (tests + window A/B), and bs=1 int4 decode
# FETCH / WRITE passes at position ~80 (prompt 80: the decode attention's K/V traffic vs the bytes
# the step uses, the dominant GEMV's traffic) summarized into gpurun_out/r04l_pmc.json.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04l
mkdir -p $O
cd $R
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 840 python -u -m pytest tests -m gpu -q --timeout 280 --timeout-method thread -p no:cacheprovider > $O/t_all.log 2>&1
chk "gpu tests" $?
LLJ_LIB=$R/scratch/w4wide.so timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -q --timeout 120 --timeout-method thread > $O/t_wide.log 2>&1
chk "w4 wide gemm tests" $?
for rep in 1 2; do
  for cfg in "X=0" "LLJ_GEMM_GLDS=1" "LLJ_LIB=$R/scratch/w4wide.so"; do
    echo "== rep $rep $cfg" >> $O/prefill_bench.log
    env $cfg timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 --iters 5 >> $O/prefill_bench.log 2>&1
    chk "prefill bench $cfg" $?
  done
done
for rep in 1 2; do
  for sp in half full; do
    echo "== rep $rep LLJ_ATT_SPEC=$sp" >> $O/decode_ab.log
    LLJ_ATT_SPEC=$sp timeout -k 10 200 python -u bench.py --decode-only --steps 300 --warmup 20 >> $O/decode_ab.log 2>&1
    chk "decode $sp" $?
  done
done
D=/tmp/r04l
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
SHORT="--steps 4 --warmup 1 --no-bs8 --no-c4 --no-cpu-baseline --eager --prompt-len 80"
for pass in FETCH_SIZE WRITE_SIZE; do
  tag=bs1_$(echo $pass | tr 'A-Z' 'a-z' | cut -d_ -f1)
  timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv -d $D -o $tag -- python3 $R/bench.py $SHORT > $D/$tag.log 2>&1
  chk "pmc $pass" $?
done
find $D -mindepth 2 -name "*counter_collection.csv" -exec mv {} $D/ \;
python3 $R/tools/profile_summary.py $D $R/gpurun_out/r04l_pmc.json >> $O/status.log 2>&1
exit 0
