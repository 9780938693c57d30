"""Build the in-tree HIP library (`_lljamd.so`) for gfx950 with hipcc. No torch in the ABI,
so a plain `hipcc -shared` is enough; the .so lives next to this file so it travels with the
repository snapshot to the GPU box."""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG.parent / "csrc"
INCLUDE = PKG.parent.parent / "include"  # the public C ABI header (llj_layer)
OUT = PKG / "_lljamd.so"
ARCH = os.environ.get("LLJ_OFFLOAD_ARCH", "gfx950")


def sources():
    return sorted(CSRC.glob("*.hip"))


def needs_build() -> bool:
    if not OUT.exists():
        return True
    t = OUT.stat().st_mtime
    return any(p.stat().st_mtime > t for p in list(CSRC.glob("*")) + [INCLUDE / "lit_llama_amd.h"])


def build(force: bool = False, verbose: bool = False) -> Path:
    if not force and not needs_build():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmp = OUT.with_suffix(".so.tmp")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall",
           "-Wno-unused-variable", "-Wno-unused-function", "-munsafe-fp-atomics", f"-I{INCLUDE}", "-o", str(tmp)] + [str(s) for s in sources()]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
