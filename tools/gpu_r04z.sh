#!/bin/bash
# Round-4 batch Z: the default bench line on the final tree with the final committed traces in place.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04z
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
echo "bench rc=$?" >> $O/status.log
exit 0
