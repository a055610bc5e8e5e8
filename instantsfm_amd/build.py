"""Build the in-tree HIP library for gfx950 (hipcc cross-compiles without a GPU).

Each source compiles to its own object under build/ (rebuilt when it or any header is newer), then one link step
produces instantsfm_amd/_lib/libinsfm_ba.so.
"""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", n) for n in ("ba_kernels.hip", "passes.hip", "tracks.hip")]
HEADERS = [*sorted(glob.glob(os.path.join(HERE, "csrc", "*.h"))), *sorted(glob.glob(os.path.join(REPO, "include", "*.h")))]
OBJDIR = os.path.join(REPO, "build", "obj")
OUT = os.path.join(HERE, "_lib", "libinsfm_ba.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics", "-Wall"]


def _obj(src):
    return os.path.join(OBJDIR, os.path.basename(src) + ".o")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def needs_build():
    return _stale(OUT, SRCS + HEADERS)


def build(force=False, verbose=True):
    os.makedirs(OBJDIR, exist_ok=True)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    procs = []
    for src in SRCS:
        obj = _obj(src)
        if force or _stale(obj, [src] + HEADERS):
            cmd = [HIPCC, f"--offload-arch={ARCH}", *FLAGS, "-c", "-o", obj + ".tmp", src]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            procs.append((subprocess.Popen(cmd), obj))
    for p, obj in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, f"hipcc {obj}")
        os.replace(obj + ".tmp", obj)
    if procs or force or _stale(OUT, [_obj(s) for s in SRCS]):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT + ".tmp", *[_obj(s) for s in SRCS]]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
