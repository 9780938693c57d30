"""Per-kernel resource usage (VGPRs, AGPRs, scratch, occupancy) of one csrc/*.hip translation unit,
from hipcc's -Rpass-analysis=kernel-resource-usage remarks (build-time check, no GPU).

  python tools/kres.py gemv_w4.hip [filter-regex]
"""
import re
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
src = REPO / "lit-llama-ja_amd" / "csrc" / sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
                      f"-I{REPO / 'include'}", "-c", str(src), "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs Spill): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0] + ("_spill" if "Spill" in m.group(1) else "")] = int(m.group(2))
for r in rows:
    n = r["name"]
    m = re.search(r"gemv_kernelI((?:Li-?\d+E)+)E", n)
    short = "gemv<" + ",".join(re.findall(r"Li(-?\d+)E", m.group(1))) + ">" if m else n
    if pat and not pat.search(short):
        continue
    print(f"{short:32s} vgpr {r.get('VGPRs', '?'):>4} agpr {r.get('AGPRs', '?'):>3} scratch {r.get('ScratchSize', '?'):>4} "
          f"occ {r.get('Occupancy', '?')}")
