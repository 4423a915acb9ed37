"""Build libzchunk.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libzchunk.so")
SOURCES = [os.path.join(CSRC, "zc_kernels.hip"), os.path.join(CSRC, "zc_engine.cpp"),
           os.path.join(CSRC, "zc_sha256.cpp"), os.path.join(CSRC, "zc_lzo.hip")]
# host-only sources (no device code; built by the host compiler with x86 intrinsics)
HOST_ONLY = {"zc_sha256.cpp"}
HEADERS = [os.path.join(CSRC, "zc_device.h"), os.path.join(CSRC, "zc_lzo_core.h"),
           os.path.join(ROOT, "include", "zchunk.h")]
ARCH = os.environ.get("ZC_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.isabs(cand) and os.path.exists(cand) or not os.path.isabs(cand)):
            return cand
    return "hipcc"


def stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in SOURCES + HEADERS)


def build(force=False, verbose=False):
    if not force and not stale():
        return LIB
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(CSRC, os.path.basename(src) + ".o")
        cmd = [hipcc(), "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
               "-I" + os.path.join(ROOT, "include"), "-c", src, "-o", obj]
        if os.path.basename(src) in HOST_ONLY:
            cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-Wall", "-I" + os.path.join(ROOT, "include"),
                   "-c", src, "-o", obj]
        elif src.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd), cmd))  # the sources compile in parallel
        objs.append(obj)
    for p, cmd in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB] + objs
    subprocess.run(cmd, check=True)
    for o in objs:
        os.remove(o)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
