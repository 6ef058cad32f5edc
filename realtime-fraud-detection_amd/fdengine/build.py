"""In-tree build of the native pieces (no cmake): hipcc for libfdengine.so (gfx950), gcc for the
CPU oracle used by tests and the bench's cpu_baseline leg.

Outputs stay in-tree (git-ignored, but shipped to the GPU box by gpurun):
  realtime-fraud-detection_amd/lib/libfdengine.so
  oracle/build/liboracle.so
"""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent
REPO_ROOT = PKG_ROOT.parent
CSRC = PKG_ROOT / "csrc"
LIB_DIR = PKG_ROOT / "lib"
ORACLE_DIR = REPO_ROOT / "oracle"

HIP_SOURCES = ["engine.hip", "forest.hip", "ensemble.hip", "blend.hip", "features.hip", "route.hip", "lstm.hip",
               "windows.hip", "snapshot.hip", "ingest.hip", "sink.hip", "model_io.hip"]
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-Wno-unused-result"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build libfdengine.so)")


def _stale(out: Path, inputs) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(p).stat().st_mtime > t for p in inputs)


def build_engine(force: bool = False, verbose: bool = True, profile: bool = False) -> Path:
    """One object per translation unit (compiled in parallel, rebuilt only when stale), then one link.
    profile=True builds lib/libfdengine_prof.so with the forest and feature kernels' phase-cycle
    instrumentation (-DFD_FOREST_PROFILE; tools/forest_phases.py / tools/feat_phases.py load it via
    FDENGINE_LIB)."""
    from concurrent.futures import ThreadPoolExecutor
    LIB_DIR.mkdir(exist_ok=True)
    obj_dir = LIB_DIR / ("obj_prof" if profile else "obj")
    obj_dir.mkdir(exist_ok=True)
    out = LIB_DIR / ("libfdengine_prof.so" if profile else "libfdengine.so")
    srcs = [CSRC / s for s in HIP_SOURCES if (CSRC / s).exists()]
    headers = list(CSRC.glob("*.h")) + [REPO_ROOT / "include" / "fdengine.h"]
    extra = ["-DFD_FOREST_PROFILE"] if profile else []
    compile_flags = [f for f in HIPCC_FLAGS if f != "-shared"]
    if not force and not _stale(out, [*srcs, *headers]):
        return out  # (the GPU box gets the library without the objects)

    def obj(src: Path) -> Path:
        o = obj_dir / (src.stem + ".o")
        if force or _stale(o, [src, *headers]):
            tmp = o.with_suffix(".o.tmp")
            cmd = [_hipcc(), *compile_flags, *extra, f"-I{REPO_ROOT / 'include'}", f"-I{CSRC}", "-c", str(src),
                   "-o", str(tmp)]
            if verbose:
                print("[build]", " ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed on {src.name}:\n{r.stderr[-6000:]}")
            tmp.replace(o)
        return o

    jobs = max(1, min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(obj, srcs))
    if not force and not _stale(out, objs):
        return out
    tmp = out.with_suffix(".so.tmp")
    cmd = [_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    tmp.replace(out)
    return out


def build_oracle(force: bool = False, verbose: bool = True) -> Path:
    bdir = ORACLE_DIR / "build"
    bdir.mkdir(exist_ok=True)
    out = bdir / "liboracle.so"
    srcs = sorted(ORACLE_DIR.glob("*.c"))
    deps = srcs + sorted(ORACLE_DIR.glob("*.h"))
    if not force and not _stale(out, deps):
        return out
    tmp = out.with_suffix(".so.tmp")
    cmd = ["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-fopenmp", "-ffp-contract=off",
           "-fno-fast-math", *map(str, srcs), "-o", str(tmp), "-lm"]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    tmp.replace(out)
    return out


def build_all(force: bool = False, verbose: bool = True) -> None:
    build_engine(force=force, verbose=verbose)
    build_oracle(force=force, verbose=verbose)


if __name__ == "__main__":
    import sys
    build_all(force="--force" in sys.argv)
    if "--profile" in sys.argv:
        build_engine(force="--force" in sys.argv, profile=True)
