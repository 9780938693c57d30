#!/bin/bash
# SQ counter passes over the persistent engine (tools/engine_probe.py: consumers alone x3, real
# steps x3, loader alone x3, eager), one pass per counter group under its own kill timeout; the
# per-dispatch rows of engine_step_kernel summarized into gpurun_out/$1.json.
OUT=$1
R=$GRAFT_REPO_ROOT
D=/tmp/$OUT
mkdir -p $D $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
run() {  # tag counters
  timeout -s KILL 150 rocprofv3 --pmc $2 --output-format csv -d $D -o $1 -- python3 $R/tools/engine_probe.py > $D/$1.log 2>&1
  echo "$1 rc=$?"
}
run eng_sqa "SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,GRBM_GUI_ACTIVE"
run eng_sqb "SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_INSTS_VMEM_RD"
run eng_sqc "SQ_VALU_MFMA_BUSY_CYCLES,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_MISC,SQ_INSTS_BRANCH,SQ_INSTS_VMEM_WR,GRBM_GUI_ACTIVE"
find $D -mindepth 2 -name "*.csv" -exec mv {} $D/ \; 2>/dev/null
cp $D/*.log $R/gpurun_out/ 2>/dev/null
python3 - "$D" "$R/gpurun_out/$OUT.json" <<'PY'
import csv, json, sys, collections
from pathlib import Path
d, out = Path(sys.argv[1]), sys.argv[2]
res = {}
for f in sorted(d.glob("*counter_collection.csv")):
    rows = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "engine_step_kernel" not in r["Kernel_Name"]:
            continue
        rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = rows[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    res[f.name] = [dict(dispatch=k, **v) for k, v in sorted(rows.items())]
Path(out).write_text(json.dumps(res, indent=1))
print("summary", out, {k: len(v) for k, v in res.items()})
PY
