#!/bin/bash
# Round-5 batch AF: rocprofv3 kernel trace + stats of the default bench command (the final build).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05af
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench.py > $O/bench.json 2> $O/bench.err
echo "prof bench rc=$?" >> $O/status.log
exit 0
