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


def src_hash() -> str:
    """Content hash of the library sources (csrc/ and include/*.h), 16 hex digits: compiled into
    the library (mlff_build_hash) so that a loaded binary can be tied to the tree it claims to be
    built from (bench.py checks it before reporting PMC traffic collected on these sources)."""
    import hashlib

    h = hashlib.sha256()
    files = sorted(list(CSRC.glob("*")) + list((REPO / "include").glob("*.h")))
    for f in files:
        if f.is_file():
            h.update(f.relative_to(REPO).as_posix().encode())
            h.update(f.read_bytes())
    return h.hexdigest()[:16]


def _hash_object(force: bool) -> Path:
    """build/obj/build_hash.o: mlff_build_hash() returning src_hash(); rewritten and recompiled
    only when the hash changes."""
    src = OBJ / "build_hash.cpp"
    obj = OBJ / "build_hash.o"
    text = ('extern "C" const char *mlff_build_hash(void) { return "%s"; }\n' % src_hash())
    if force or not src.exists() or src.read_text() != text or not obj.exists():
        src.write_text(text)
        cmd = [HIPCC, "-O2", "-fPIC", "-x", "c++", "-c", str(src), "-o", str(obj)]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"hipcc failed for build_hash.cpp:\n{res.stdout}\n{res.stderr}")
    return obj


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
    objs.append(_hash_object(force))
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
