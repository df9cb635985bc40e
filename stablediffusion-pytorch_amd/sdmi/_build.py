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
ARCH = "gfx950"
# per-source extra flags. attention.hip: softmax maxima are taken straight from MFMA accumulators; in the default
# IEEE mode every fmaxf input would first be quieted by a canonicalising v_max_f32 (one extra VALU op per score).
# The kernels never produce or consume NaNs (masked scores are -inf), so IEEE mode is switched off there.
# -fno-slp-vectorize: the softmax VALU is written as scalar f32 ops; SLP would re-pack adjacent ones into
# v_pk_{fma,mul,add}_f32, which beside MFMAs cost about three times two scalar ops (MI355X guide, 'price of one
# filler beside MFMAs').
EXTRA_FLAGS = {"attention.hip": ["-fno-honor-nans", "-mno-amdgpu-ieee", "-fno-slp-vectorize"],
               # gemm.hip: the VALU bias row sums of the weight-gradient mainloop run beside the MFMAs (same reason)
               "gemm.hip": ["-fno-slp-vectorize"]}


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps += [os.path.join(REPO, "include", "sdmi.h"), os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False, out=None, defines=()):
    """out / defines: a probe variant of the library (e.g. SDMI_GEMM_TRACE into libsdmi_trace.so), loaded through
    SDMI_LIB_PATH by scripts only -- never the product library."""
    lib_out = out or LIB
    if not force and out is None and not needs_build():
        return LIB
    objs = []
    procs = []
    for src in sources():
        obj = os.path.join("/tmp", "sdmi_" + os.path.basename(src) + f".{os.getpid()}.o")
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj,
               "-I", os.path.join(REPO, "include"), "-Rpass-analysis=kernel-resource-usage"]
        cmd += EXTRA_FLAGS.get(os.path.basename(src), [])
        cmd += [f"-D{d}" for d in defines]
        procs.append((subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT), src, cmd))
        objs.append(obj)
    spills = []
    for p, src, cmd in procs:
        out, _ = p.communicate()
        txt = out.decode(errors="replace")
        if p.returncode != 0:
            sys.stderr.write(txt)
            raise RuntimeError(f"hipcc failed on {src}")
        # guard: no kernel may use scratch for VGPR spills or private arrays (silent 3x slowdowns). A few
        # SGPR spills that overflow into scratch (epilogue-only argument pressure) are tolerated.
        usage = {}
        fn = None
        for line in txt.splitlines():
            if "Function Name:" in line:
                fn = line.split("Function Name:")[1].split("[")[0].strip()
                usage[fn] = {}
            elif fn is not None:
                for key in ("ScratchSize [bytes/lane]:", "VGPRs Spill:", "SGPRs Spill:"):
                    if key in line:
                        usage[fn][key] = int(line.split(key)[1].split("[")[0])
        for fn, u in usage.items():
            scratch = u.get("ScratchSize [bytes/lane]:", 0)
            sgpr_only = u.get("VGPRs Spill:", 0) == 0 and u.get("SGPRs Spill:", 0) > 0 and scratch <= 64
            if scratch > 0 and not sgpr_only:
                spills.append((os.path.basename(src), fn, scratch))
        if verbose:
            sys.stderr.write("\n".join(l for l in txt.splitlines() if "remark" not in l))
    if spills:
        raise RuntimeError(f"kernels use scratch memory (register spill / dynamic indexing): {spills}")
    tmp = lib_out + f".tmp{os.getpid()}"
    subprocess.check_call(["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs)
    os.replace(tmp, lib_out)
    for o in objs:
        try:
            os.remove(o)
        except OSError:
            pass
    return lib_out


def source_digest():
    """16-hex-digit sha256 over the library's sources (csrc/*.hip, csrc/*.h, include/sdmi.h, by name) and the tuned
    GEMM table (sdmi/tuned_gemm.json: its split counts set every launch's grid and slab traffic): the tree a
    committed profile (profiles/rNN_<workload>_pmc_traffic.json / _roofline_evidence.json) was measured on. bench.py
    compares it with the running tree's, so a stale PMC file is reported as such instead of silently reused."""
    import hashlib
    h = hashlib.sha256()
    files = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".h")))
    for f in files:
        h.update(f.encode())
        h.update(open(os.path.join(CSRC, f), "rb").read())
    h.update(open(os.path.join(REPO, "include", "sdmi.h"), "rb").read())
    h.update(open(os.path.join(HERE, "tuned_gemm.json"), "rb").read())
    return h.hexdigest()[:16]


CABI_SRC = os.path.join(REPO, "tests", "cabi", "cabi_check.c")
CABI_BIN = os.path.join(REPO, "tests", "cabi", "cabi_check")


def build_cabi_check():
    """The plain-C caller of include/sdmi.h (tests/cabi/cabi_check.c), compiled by gcc as C against libsdmi.so and the
    HIP runtime: proves the boundary is callable without PyTorch or C++ (tests/test_cabi_gpu.py runs it)."""
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    tmp = CABI_BIN + f".tmp{os.getpid()}"
    subprocess.check_call(["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                           "-I", os.path.join(rocm, "include"), "-I", os.path.join(REPO, "include"), CABI_SRC,
                           "-o", tmp, "-L", HERE, "-lsdmi", "-L", os.path.join(rocm, "lib"), "-lamdhip64",
                           "-Wl,-rpath,$ORIGIN/../../stablediffusion-pytorch_amd/sdmi",
                           "-Wl,-rpath," + os.path.join(rocm, "lib")])
    os.replace(tmp, CABI_BIN)
    return CABI_BIN


if __name__ == "__main__":
    if "--digest" in sys.argv:
        print(source_digest())
    elif "--trace" in sys.argv:  # the GEMM phase-timestamp probe library (scripts/gemm_phase_probe.py)
        print(build(force=True, out=os.path.join(HERE, "libsdmi_trace.so"), defines=("SDMI_GEMM_TRACE",)))
    else:
        print(build(force="--force" in sys.argv, verbose=True))
