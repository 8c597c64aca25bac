#!/usr/bin/env python3
"""Build an alternative copy of the package for same-box A/B runs (CPU side, before a gpurun call).

    python3 scripts/mi355x/ab_build.py <name> <patch-file | -> [--rev REV]

Checks out REV (default HEAD) of the source tree into /tmp/ab_<name>/src, applies the patch (a `git diff` of
csrc/...; `-` for none), builds it with the same CMake options as stencil2_amd._build, and installs the Python
package with its freshly built .so files into lab_alt/<name>/stencil2_amd (git-ignored, shipped to the box by
gpurun). On the box: PYTHONPATH=lab_alt/<name> python3 scripts/mi355x/shape_sweep.py ... runs the alternative.
"""
import argparse
import glob
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("name")
ap.add_argument("patch")
ap.add_argument("--rev", default="HEAD")
ap.add_argument("--jobs", type=int, default=8)
args = ap.parse_args()

work = f"/tmp/ab_{args.name}"
src, bld = os.path.join(work, "src"), os.path.join(work, "build")
if os.path.exists(src):
    shutil.rmtree(src)
os.makedirs(src)
subprocess.run(f"git -C {REPO} archive {args.rev} | tar -x -C {src}", shell=True, check=True)
if args.patch != "-":
    subprocess.run(["git", "apply", os.path.abspath(args.patch)], cwd=src, check=True)
if not os.path.exists(os.path.join(bld, "build.ninja")):
    subprocess.run(["cmake", "-S", src, "-B", bld, "-G", "Ninja", "-DCMAKE_HIP_ARCHITECTURES=gfx950",
                    "-DCMAKE_BUILD_TYPE=Release", f"-DPython3_EXECUTABLE={sys.executable}"], check=True,
                   stdout=subprocess.DEVNULL, env=dict(os.environ, CMAKE_PREFIX_PATH="/opt/rocm"))
subprocess.run(["cmake", "--build", bld, "-j", str(args.jobs), "--target", "_C", "stencil2"], check=True,
               stdout=subprocess.DEVNULL)
dst = os.path.join(REPO, "lab_alt", args.name, "stencil2_amd")
if os.path.exists(dst):
    shutil.rmtree(dst)
shutil.copytree(os.path.join(src, "stencil2_amd"), dst)
for so in glob.glob(os.path.join(bld, "_C*.so")) + [os.path.join(bld, "libstencil2.so")]:
    shutil.copy2(so, dst)
print("installed", dst)
