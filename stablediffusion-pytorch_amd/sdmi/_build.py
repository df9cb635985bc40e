"""Builds libsdmi.so (all HIP kernels + the C ABI of include/sdmi.h) in-tree for gfx950.

The shared library is compiled with plain hipcc (no torch headers): the boundary is a C ABI and
Python binds it with ctypes (sdmi/_lib.py)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
CSRC = os.path.join(PKG, "csrc")
REPO = os.path.dirname(PKG)
LIB = os.path.join(HERE, "libsdmi.so")
ARCH = os.environ.get("SDMI_ARCH", "gfx950")


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps.append(os.path.join(REPO, "include", "sdmi.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    if not force and not needs_build():
        return LIB
    objs = []
    procs = []
    for src in sources():
        obj = os.path.join("/tmp", "sdmi_" + os.path.basename(src) + f".{os.getpid()}.o")
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj,
               "-I", os.path.join(REPO, "include")]
        procs.append((subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT), src, cmd))
        objs.append(obj)
    for p, src, cmd in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(out.decode())
            raise RuntimeError(f"hipcc failed on {src}")
        if verbose and out:
            sys.stderr.write(out.decode())
    tmp = LIB + f".tmp{os.getpid()}"
    subprocess.check_call(["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs)
    os.replace(tmp, LIB)
    for o in objs:
        try:
            os.remove(o)
        except OSError:
            pass
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
