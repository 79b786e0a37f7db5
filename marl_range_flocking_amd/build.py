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


def build(force=False, verbose=False):
    if not force and not _stale():
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
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
