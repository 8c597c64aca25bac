"""In-tree build of the native runtime (CMake + Ninja, hipcc for gfx950).

Produces ``stencil2_amd/_C*.so`` (pybind11 module) and ``stencil2_amd/libstencil2.so`` (the C++/HIP runtime),
plus the C++ apps in ``build/bin``. Everything stays in-tree so it travels with a gpurun snapshot.
"""
from __future__ import annotations

import glob
import hashlib
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "stencil2_amd")
BUILD = os.path.join(REPO, "build")


def _sources():
    pats = ["csrc/**/*.hpp", "csrc/**/*.cpp", "csrc/**/*.hip", "CMakeLists.txt", "cmake/*.cmake"]
    out = []
    for p in pats:
        out += glob.glob(os.path.join(REPO, p), recursive=True)
    return out


def _artifacts():
    return glob.glob(os.path.join(PKG, "_C*.so")) + glob.glob(os.path.join(PKG, "libstencil2.so"))


STAMP = os.path.join(PKG, ".build_stamp")


def _source_hash() -> str:
    """sha256 over the native sources' paths and contents: copies, checkouts and snapshots change mtimes without
    changing what the artifacts were built from"""
    h = hashlib.sha256()
    for f in sorted(_sources()):
        h.update(os.path.relpath(f, REPO).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def is_stale() -> bool:
    arts = _artifacts()
    if len(arts) < 2 or not os.path.exists(os.path.join(BUILD, "bin", "jacobi3d")):
        return True
    if os.path.exists(STAMP):
        with open(STAMP) as f:
            return f.read().strip() != _source_hash()
    newest_src = max(os.path.getmtime(s) for s in _sources())
    oldest_art = min(os.path.getmtime(a) for a in arts)
    return newest_src > oldest_art


def build(verbose: bool = False, jobs: int | None = None) -> None:
    """Configure (once) and build everything; copy the Python-facing .so files into the package."""
    jobs = jobs or min(8, os.cpu_count() or 8)
    env = dict(os.environ)
    env.setdefault("CMAKE_PREFIX_PATH", "/opt/rocm")
    if not os.path.exists(os.path.join(BUILD, "build.ninja")):
        os.makedirs(BUILD, exist_ok=True)
        cmd = ["cmake", "-S", REPO, "-B", BUILD, "-G", "Ninja", "-DCMAKE_HIP_ARCHITECTURES=gfx950",
               "-DCMAKE_BUILD_TYPE=Release", f"-DPython3_EXECUTABLE={sys.executable}"]
        subprocess.run(cmd, check=True, env=env, stdout=None if verbose else subprocess.DEVNULL)
    r = subprocess.run(["ninja", "-C", BUILD, f"-j{jobs}"], env=env, capture_output=not verbose, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + (r.stdout or "")[-8000:] + (r.stderr or "")[-4000:])
    for so in glob.glob(os.path.join(BUILD, "_C*.so")) + [os.path.join(BUILD, "libstencil2.so")]:
        dst = os.path.join(PKG, os.path.basename(so))
        tmp = dst + ".tmp"
        shutil.copy2(so, tmp)
        os.replace(tmp, dst)
    with open(STAMP + ".tmp", "w") as f:
        f.write(_source_hash() + "\n")
    os.replace(STAMP + ".tmp", STAMP)


def ensure_built() -> None:
    if not is_stale():
        return
    if _artifacts() and not os.path.exists(os.path.join(BUILD, "CMakeFiles", "rules.ninja")):
        # a snapshot without the configured build tree (a GPU box): the shipped artifacts were built from other
        # sources than these. Loading them would run stale native code under tests and benchmarks, so refuse unless
        # explicitly allowed.
        msg = ("stencil2_amd: the native sources differ from the build stamp and no build tree is configured here; "
               "rebuild in-tree (python -m stencil2_amd._build) before shipping")
        if os.environ.get("STENCIL_ALLOW_STALE") == "1":
            print(msg + " -- loading the shipped artifacts anyway (STENCIL_ALLOW_STALE=1)", file=sys.stderr)
            return
        raise RuntimeError(msg + " (or set STENCIL_ALLOW_STALE=1 to load the stale artifacts)")
    build()


if __name__ == "__main__":
    build(verbose="-v" in sys.argv)
    print("built:", _artifacts())
