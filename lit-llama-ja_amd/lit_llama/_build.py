"""Build the in-tree HIP library (`_lljamd.so`) for gfx950 with hipcc. No torch in the ABI,
so plain `hipcc` objects linked with `-shared` are enough; the .so lives next to this file so
it travels with the repository snapshot to the GPU box. The translation units compile in
parallel (one hipcc per .hip file), then link."""
from __future__ import annotations

import os
import subprocess
import tempfile
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG.parent / "csrc"
INCLUDE = PKG.parent.parent / "include"  # the public C ABI header (llj_layer)
OUT = PKG / "_lljamd.so"
ARCH = os.environ.get("LLJ_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-variable", "-Wno-unused-function",
         "-munsafe-fp-atomics"]


# per-file flags: the GPTQ column loop reproduces the reference's fp32 op order bit for bit, so
# no multiply-add contraction there (hipcc contracts by default and ignores the fp pragma)
FILE_FLAGS = {"gptq.hip": ["-ffp-contract=off"]}


def sources():
    return sorted(CSRC.glob("*.hip"))


def needs_build() -> bool:
    if not OUT.exists():
        return True
    t = OUT.stat().st_mtime
    return any(p.stat().st_mtime > t for p in list(CSRC.glob("*")) + [INCLUDE / "lit_llama_amd.h"])


OBJ_CACHE = PKG.parent.parent / "build" / "obj"  # per-source objects of the in-tree library (git-ignored)


def _stale(obj: Path, src: Path) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    deps = [src] + list(CSRC.glob("*.h")) + [INCLUDE / "lit_llama_amd.h", Path(__file__)]
    return any(d.stat().st_mtime > t for d in deps)


def build(force: bool = False, verbose: bool = False, out: Path | None = None, defines=()) -> Path:
    """Compile every csrc/*.hip for gfx950 and link `out` (default: the in-tree _lljamd.so).
    `defines`: extra -D macros (profiling / experiment variants built next to the product).
    The product build keeps one object per source under build/obj and recompiles only the sources
    whose file (or any shared header) changed; force=True recompiles everything."""
    out = Path(out) if out is not None else OUT
    if out == OUT and not defines and not force and not needs_build():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    extra = [f"-D{d}" for d in defines]
    with tempfile.TemporaryDirectory(prefix="lljbuild") as td:
        cache = OBJ_CACHE if (out == OUT and not defines) else Path(td)
        cache.mkdir(parents=True, exist_ok=True)
        objs = []
        cmds = []
        for src in sources():
            obj = cache / (src.stem + ".o")
            objs.append(obj)
            if force or cache != OBJ_CACHE or _stale(obj, src):
                cmds.append([hipcc, f"--offload-arch={ARCH}", *FLAGS, *FILE_FLAGS.get(src.name, []), *extra,
                             f"-I{INCLUDE}", "-c", str(src), "-o", str(obj)])

        def run(cmd):
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)

        if cmds:
            with ThreadPoolExecutor(max_workers=min(len(cmds), 8)) as ex:
                list(ex.map(run, cmds))
        tmp = out.with_suffix(".so.tmp")
        link = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp)] + [str(o) for o in objs]
        run(link)
        os.replace(tmp, out)
    return out


if __name__ == "__main__":
    import sys

    args = sys.argv[1:]
    o = Path(args[0]) if args else None
    print(build(force=True, verbose=True, out=o, defines=args[1:]))
