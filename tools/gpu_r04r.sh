#!/bin/bash
# Round-4 batch R: bs=1 int4 decode FETCH / WRITE passes at position ~80 on the final tree (decode
# attention 512 x 4), summarized into gpurun_out/r04r_pmc.json (tools/profile_summary.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04r
mkdir -p $O
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
D=/tmp/r04r
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
SHORT="--steps 4 --warmup 1 --no-bs8 --no-c4 --no-cpu-baseline --eager --prompt-len 80"
for pass in FETCH_SIZE WRITE_SIZE; do
  tag=bs1_$(echo $pass | tr 'A-Z' 'a-z' | cut -d_ -f1)
  timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv -d $D -o $tag -- python3 $R/bench.py $SHORT > $D/$tag.log 2>&1
  chk "pmc $pass" $?
done
find $D -mindepth 2 -name "*counter_collection.csv" -exec mv {} $D/ \;
python3 $R/tools/profile_summary.py $D $R/gpurun_out/r04r_pmc.json >> $O/status.log 2>&1
exit 0
