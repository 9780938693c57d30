"""Experiment variants of the HIP library for A/B runs (tools/ab_decode.py LIB=...): the listed
translation units recompiled with extra -D macros, linked with the product's cached objects
(build/obj, from lit_llama._build) for the rest. Not the product .so.

  python tools/build_variant.py scratch/drm3.so LLJ_DRM=3 --tu gemv_w4 gemv_w8 gemv_bf16 gemv_w4g
"""
from __future__ import annotations

import argparse
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "lit-llama-ja_amd"))
from lit_llama import _build  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("defines", nargs="*")
    ap.add_argument("--tu", nargs="+", required=True, help="translation units (csrc/<name>.hip) to recompile")
    a = ap.parse_args()
    _build.build()  # the product objects are current
    out = Path(a.out)
    if not out.is_absolute():
        out = REPO / out
    od = out.parent / ("obj_" + out.stem)
    od.mkdir(parents=True, exist_ok=True)
    hipcc = "/opt/rocm/bin/hipcc"
    objs, cmds = [], []
    for src in _build.sources():
        if src.stem in a.tu:
            o = od / (src.stem + ".o")
            cmds.append([hipcc, f"--offload-arch={_build.ARCH}", *_build.FLAGS, *_build.FILE_FLAGS.get(src.name, []),
                         *[f"-D{d}" for d in a.defines], f"-I{_build.INCLUDE}", "-c", str(src), "-o", str(o)])
            objs.append(o)
        else:
            objs.append(_build.OBJ_CACHE / (src.stem + ".o"))
    with ThreadPoolExecutor(max_workers=8) as ex:
        list(ex.map(lambda c: subprocess.run(c, check=True), cmds))
    subprocess.run([hipcc, f"--offload-arch={_build.ARCH}", "-shared", "-fPIC", "-o", str(out)] + [str(o) for o in objs],
                   check=True)
    print(out)


if __name__ == "__main__":
    main()
