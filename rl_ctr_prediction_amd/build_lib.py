"""Build libctr_hip.so (gfx950) in-tree with hipcc.

Each source compiles to an object in ``build/`` (in parallel), then one shared library is
linked next to this file so it travels to the GPU box with the repo snapshot. Objects
are rebuilt only when a source or header is newer. Run ``python -m
rl_ctr_prediction_amd.build_lib`` or call :func:`build`.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = ROOT / "build" / "ctr_hip"
LIB = PKG / "libctr_hip.so"
ARCH = os.environ.get("CTR_OFFLOAD_ARCH", "gfx950")

SOURCES = ["abi.cpp", "fm_forward.hip", "sparse_plan.hip", "sparse_grad.hip", "adam.hip",
           "gemm.hip", "gemm_sb16.hip", "gemm_planes.hip", "reduce_pg.hip", "pnn.hip", "io.cpp", "ensemble.hip", "ffm.hip",
           "layout.hip", "ops.hip"]
INCLUDE_DIRS = [CSRC, ROOT / "include"]

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
            "-Wall", "-Wno-unused-function", "-I", str(ROOT / "include")]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain (ROCm) is required to build "
                       "libctr_hip.so")


def _deps(src: Path, seen: set | None = None) -> set:
    """src and every local header it includes, transitively (`#include "..."` lines
    resolved against the source's directory, csrc/ and include/)."""
    seen = set() if seen is None else seen
    if src in seen:
        return seen
    seen.add(src)
    for line in src.read_text(errors="replace").splitlines():
        line = line.strip()
        if not line.startswith("#include") or '"' not in line:
            continue
        name = line.split('"')[1]
        for d in [src.parent, *INCLUDE_DIRS]:
            h = d / name
            if h.exists():
                _deps(h.resolve(), seen)
                break
    return seen


def _stale(obj: Path, src: Path) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(p.stat().st_mtime > t for p in _deps(src.resolve()))


def _compile(hipcc: str, src: Path, obj: Path) -> None:
    cmd = [hipcc, *CXXFLAGS, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")


def build(verbose: bool = False, jobs: int = 6) -> Path:
    hipcc = _hipcc()
    BUILD.mkdir(parents=True, exist_ok=True)
    todo = []
    objs = []
    for name in SOURCES:
        src = CSRC / name
        obj = BUILD / (name.rsplit(".", 1)[0] + ".o")
        objs.append(obj)
        if _stale(obj, src):
            todo.append((src, obj))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            futs = {ex.submit(_compile, hipcc, s, o): s for s, o in todo}
            for f in cf.as_completed(futs):
                f.result()
                if verbose:
                    print(f"[build] compiled {futs[f].name}", flush=True)
    if todo or not LIB.exists() or any(o.stat().st_mtime > LIB.stat().st_mtime for o in objs):
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp),
               *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
        if verbose:
            print(f"[build] linked {LIB}", flush=True)
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
