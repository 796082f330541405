"""Build libmlffpcg.so (HIP for gfx950) in-tree.

    python mlff-preconditioner_amd/build_native.py [--force] [--jobs N]

Compiles every csrc/*.hip with hipcc --offload-arch=gfx950 and links them with
RCCL into mlff-preconditioner_amd/lib/libmlffpcg.so.  Incremental: an object is
rebuilt when its source or any csrc/*.h / include/*.h is newer.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
REPO = PKG.parent
CSRC = PKG / "csrc"
OBJ = PKG / "build" / "obj"
LIB = PKG / "lib" / "libmlffpcg.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MLFF_OFFLOAD_ARCH", "gfx950")

CFLAGS = [
    "-O3",
    f"--offload-arch={ARCH}",
    "-fPIC",
    "-std=c++17",
    "-Wall",
    "-Wno-unused-function",
    "-Wno-unused-variable",
    "-I" + str(REPO / "include"),
]
LDFLAGS = ["-shared", f"--offload-arch={ARCH}", "-L/opt/rocm/lib", "-lrccl",
           "-Wl,-rpath,/opt/rocm/lib"]


def _newest_header() -> float:
    hs = list(CSRC.glob("*.h")) + list((REPO / "include").glob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _compile(src: Path, force: bool) -> Path:
    obj = OBJ / (src.stem + ".o")
    if (not force and obj.exists()
            and obj.stat().st_mtime >= max(src.stat().st_mtime, _newest_header())):
        return obj
    cmd = [HIPCC, *CFLAGS, "-c", str(src), "-o", str(obj)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{res.stdout}\n{res.stderr}")
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    LIB.parent.mkdir(parents=True, exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    if not srcs:
        raise RuntimeError("no HIP sources found")
    jobs = jobs or min(len(srcs), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if (force or not LIB.exists()
            or LIB.stat().st_mtime < max(o.stat().st_mtime for o in objs)):
        cmd = [HIPCC, *LDFLAGS, *map(str, objs), "-o", str(LIB)]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed:\n{res.stdout}\n{res.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    a = ap.parse_args()
    try:
        build(force=a.force, jobs=a.jobs)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
