#!/bin/bash
# MFMA busy of the prefill kernels (gemm_kernel, gemm_glds_kernel, flash_prefill_kernel): one rocprofv3 --pmc pass
# (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE) over one 7B 2048-token window per
# mode, summarized per kernel on the box into gpurun_out/$1.json.
#   mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
OUT=$1
MODES=${2:-gptq.int4 none}
R=$GRAFT_REPO_ROOT
D=/tmp/$OUT
mkdir -p $D $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $D -o pf \
  -- python3 $R/tools/prefill_bench.py --T 2048 --modes $MODES --iters 1 > $D/pf.log 2>&1
echo "rc=$?"
python3 - "$D" "$R/gpurun_out/$OUT.json" "$MODES" <<'PY'
import csv, glob, json, sys, collections
d, out, modes = sys.argv[1], sys.argv[2], sys.argv[3]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "gemm_kernel" not in n and "gemm_glds_kernel" not in n and "flash" not in n:
            continue
        key = n.split("(")[0].replace("void ", "")
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            cnt[key] += 1
res = {}
for k, v in agg.items():
    e = dict(v)
    e["dispatches"] = cnt[k]
    if v.get("GRBM_GUI_ACTIVE"):
        e["mfma_busy"] = v["SQ_VALU_MFMA_BUSY_CYCLES"] / (v["GRBM_GUI_ACTIVE"] / 8 * 1024)
    res[k] = e
json.dump({"what": f"rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE over tools/prefill_bench.py --T 2048 --modes {modes} --iters 1 (7B)",
           "formula": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)", "kernels": res},
          open(out, "w"), indent=1)
print(json.dumps({k: round(e.get("mfma_busy", -1), 3) for k, e in res.items()}))
PY
