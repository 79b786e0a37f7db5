"""Build libflock_amd.so in-tree with hipcc for gfx950 (no JIT cache, no pip install: the .so travels with the repo).

    python -m marl_range_flocking_amd.build [--force]
"""
import glob
import os
import shutil
import subprocess
import sys

from ._native import BUILD_DIR, LIB_PATH, PKG

ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
ARCH = os.environ.get("FLOCK_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: no FMA contraction — every float op rounds separately, as in the reference's torch op sequence.
HIPCC_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}"]


TORCH_OPS_SRCS = [os.path.join(CSRC, f) for f in ("flock_torch.cpp", "flock_torch_learn.cpp", "flock_torch_loop.cpp")]
TORCH_OPS_LIB = os.path.join(BUILD_DIR, "libflock_torch.so")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _stale():
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def hipcc():
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


# per-file extras: the env step's scan loops are written with explicit packed-f32 pairs; SLP vectorisation of the
# remaining scalar ops only adds register moves and half-rate packed ops there
FILE_FLAGS = {"flock_env.hip": ["-fno-slp-vectorize"]}


def build_torch_ops(force=False, verbose=False):
    """libflock_torch.so: the TORCH_LIBRARY(flock) custom ops (csrc/flock_torch*.cpp), host C++ over libflock_amd.so,
    compiled against this interpreter's torch headers and linked with rpath $ORIGIN."""
    deps = TORCH_OPS_SRCS + [LIB_PATH] + glob.glob(os.path.join(INCLUDE, "*.h"))
    if not force and os.path.exists(TORCH_OPS_LIB) and all(os.path.getmtime(d) <= os.path.getmtime(TORCH_OPS_LIB)
                                                           for d in deps):
        return TORCH_OPS_LIB
    import torch

    tdir = os.path.dirname(torch.__file__)
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    tmp = TORCH_OPS_LIB + ".tmp"
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}", "-I", INCLUDE,
           "-I", os.path.join(rocm, "include"), "-I", os.path.join(tdir, "include"),
           "-I", os.path.join(tdir, "include", "torch", "csrc", "api", "include"), *TORCH_OPS_SRCS, "-o", tmp,
           "-L", BUILD_DIR, "-lflock_amd", "-L", os.path.join(tdir, "lib"), "-lc10", "-lc10_hip", "-ltorch",
           "-ltorch_cpu", "-L", os.path.join(rocm, "lib"), "-lamdhip64", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(tmp, TORCH_OPS_LIB)
    return TORCH_OPS_LIB


def build(force=False, verbose=False):
    if not force and not _stale():
        build_torch_ops(False, verbose)
        return LIB_PATH
    os.makedirs(BUILD_DIR, exist_ok=True)
    objs = []
    procs = []
    for src in sources():
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        cmd = [hipcc()] + HIPCC_FLAGS + FILE_FLAGS.get(os.path.basename(src), []) + ["-c", "-I", INCLUDE, "-o", obj,
                                                                                   src]
        if verbose:
            print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    for pr in procs:
        if pr.wait() != 0:
            raise subprocess.CalledProcessError(pr.returncode, "hipcc")
    tmp = LIB_PATH + ".tmp"
    cmd = [hipcc()] + HIPCC_FLAGS + ["-shared", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(tmp, LIB_PATH)
    build_torch_ops(True, verbose)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
