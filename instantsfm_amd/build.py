"""Build the in-tree HIP library for gfx950 (hipcc cross-compiles without a GPU)."""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", "ba_kernels.hip"), os.path.join(HERE, "csrc", "passes.hip")]
DEPS = [*SRCS, *sorted(glob.glob(os.path.join(HERE, "csrc", "*.h"))), *sorted(glob.glob(os.path.join(REPO, "include", "*.h")))]
OUT = os.path.join(HERE, "_lib", "libinsfm_ba.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-munsafe-fp-atomics", "-Wall"]


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [HIPCC, f"--offload-arch={ARCH}", *FLAGS, "-o", OUT + ".tmp", *SRCS]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
