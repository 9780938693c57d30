#!/bin/bash
# round 6 batch R: the whole GPU suite, smoke and the default bench line on the current build
set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
