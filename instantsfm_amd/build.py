"""Build the in-tree HIP library for gfx950 (hipcc cross-compiles without a GPU).

Each source compiles to its own object under build/ (rebuilt when it or any header is newer), then one link step
produces instantsfm_amd/_lib/libinsfm_ba.so.
"""
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", n) for n in ("ba_kernels.hip", "passes.hip", "tracks.hip")]
HEADERS = [*sorted(glob.glob(os.path.join(HERE, "csrc", "*.h"))), *sorted(glob.glob(os.path.join(REPO, "include", "*.h")))]
OBJDIR = os.path.join(REPO, "build", "obj")
OUT = os.path.join(HERE, "_lib", "libinsfm_ba.so")
# host-side packing extension (plain C / OpenMP, CPython buffer protocol): processors/bundle_adjustment.py pack()
PACKX_SRC = os.path.join(HERE, "csrc", "packx.c")
PACKX_OUT = os.path.join(HERE, "_lib", "_packx" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics", "-Wall"]


def _obj(src):
    return os.path.join(OBJDIR, os.path.basename(src) + ".o")


def source_hash():
    """SHA-256 (first 16 hex digits) over the library's sources and headers (contents, in a fixed order): the `src=`
    field of insfm_build_info(), so a loaded library can be matched to the tree.  The target and flags it was built
    with are reported beside it (arch=, flags=) but not hashed: the load-time check compares sources only, so an
    environment that sets PYTORCH_ROCM_ARCH differently at load time does not reject an unchanged build."""
    h = hashlib.sha256()
    for path in SRCS + HEADERS:
        h.update(os.path.relpath(path, REPO).encode())
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _build_info_src():
    """A one-function source carrying the provenance string (regenerated when the hash changes)."""
    info = f"src={source_hash()} arch={ARCH} flags={' '.join(FLAGS)}"
    path = os.path.join(OBJDIR, "build_info.cpp")
    text = ('extern "C" __attribute__((visibility("default"))) const char* insfm_build_info(void) '
            f'{{ return "{info}"; }}\n')
    old = open(path).read() if os.path.exists(path) else None
    if old != text:
        with open(path, "w") as f:
            f.write(text)
    return path


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def packx_hash():
    """SHA-256 (first 16 hex digits) of csrc/packx.c: compiled into the extension as _packx.SRC_HASH and compared at
    import (processors/bundle_adjustment.py), like the main library's provenance check."""
    with open(PACKX_SRC, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def needs_build():
    return _stale(OUT, SRCS + HEADERS) or _stale(PACKX_OUT, [PACKX_SRC])


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
    info_src = _build_info_src()
    info_obj = info_src + ".o"
    if force or _stale(info_obj, [info_src]):
        subprocess.run([os.environ.get("CXX", "g++"), "-O2", "-fPIC", "-c", "-o", info_obj, info_src], check=True)
    if procs or force or _stale(OUT, [_obj(s) for s in SRCS] + [info_obj]):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT + ".tmp", *[_obj(s) for s in SRCS],
               info_obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(OUT + ".tmp", OUT)
    build_packx(force, verbose)
    return OUT


def _numpy_include():
    import numpy
    return numpy.get_include()


def build_packx(force=False, verbose=True):
    """The packing extension: no FMA contraction (its cheirality test must round like numpy's unfused operations)."""
    if not (force or _stale(PACKX_OUT, [PACKX_SRC])):
        return PACKX_OUT
    cmd = [os.environ.get("CC", "gcc"), "-O2", "-fPIC", "-shared", "-pthread", "-ffp-contract=off", "-std=gnu99",
           "-Wall", f'-DPACKX_SRC_HASH="{packx_hash()}"', f"-I{sysconfig.get_paths()['include']}",
           f"-I{_numpy_include()}", "-o", PACKX_OUT + ".tmp", PACKX_SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(PACKX_OUT + ".tmp", PACKX_OUT)
    return PACKX_OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
