"""Build the HIP library in-tree: deephall_amd/_lib/libdeephall_amd.so (gfx950).

Plain ``hipcc`` invocations (no cmake / torch JIT): each ``csrc/*.hip`` and
``csrc/*.cpp`` compiles to an object under ``build/``, then one shared library is
linked into ``deephall_amd/_lib/`` so it travels with the repository snapshot.
"""

from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
OUT_DIR = PKG / "_lib"
LIB = OUT_DIR / "libdeephall_amd.so"
ARCH = os.environ.get("DH_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-I", str(ROOT / "include")]
# per-file extras: the split-bf16 GEMM keeps its f32 subtractions scalar (packed f32 VALU
# between MFMAs costs more issue cycles than it saves, MI355X_MICROARCH.md cycle table); the
# fused channel tail likewise (round 5: the packed form of layer 1's residual spilled 44 B per
# lane; without it no spills, channel launches 440 -> 438 us, profiles/r05_v26_lnch_noslp_ab.txt)
EXTRA = {"gemm_x6.hip": ["-fno-slp-vectorize"], "gemm_lnch.hip": ["-fno-slp-vectorize"]}


def sources():
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.cpp")))


def build(verbose: bool = False, force: bool = False) -> Path:
    objdir = ROOT / "build" / ARCH
    objdir.mkdir(parents=True, exist_ok=True)
    OUT_DIR.mkdir(parents=True, exist_ok=True)
    headers = list(CSRC.glob("*.h")) + list((ROOT / "include").glob("*.h"))
    hdr_mtime = max((h.stat().st_mtime for h in headers), default=0.0)
    procs, objs = [], []
    for src in sources():
        obj = objdir / (src.name + ".o")
        objs.append(obj)
        if not force and obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, hdr_mtime):
            continue
        cmd = [HIPCC, f"--offload-arch={ARCH}", *FLAGS, *EXTRA.get(src.name, []), "-c", str(src), "-o", str(obj)]
        if src.suffix == ".cpp":
            cmd = [HIPCC, *FLAGS, "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    failed = []
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed.append((src, out.decode(errors="replace")))
        elif verbose and out:
            print(out.decode(errors="replace"), file=sys.stderr)
    if failed:
        msg = "\n".join(f"--- {s}\n{o}" for s, o in failed)
        raise RuntimeError(f"HIP build failed:\n{msg}")
    # the link manifest: a source added or removed relinks even when every object is older
    manifest = objdir / "link.manifest"
    names = "\n".join(o.name for o in objs)
    relink = (force or not LIB.exists() or any(o.stat().st_mtime > LIB.stat().st_mtime for o in objs)
              or not manifest.exists() or manifest.read_text() != names)
    if relink:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB), *map(str, objs)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        manifest.write_text(names)
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv, force="-f" in sys.argv))
