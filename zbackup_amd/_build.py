"""Build libzchunk.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
import hashlib
import os
import re
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


def source_digest():
    """sha256 over every source and header the library is built from (and the
    offload arch), first 16 hex digits: the build id libzchunk.so carries."""
    h = hashlib.sha256(ARCH.encode())
    for p in SOURCES + HEADERS:
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def lib_build_id(path=LIB):
    """The build id embedded in a built library (read from the file, without
    loading it), or None."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        m = re.search(rb"zc-build-id:([0-9a-f]{16}|unknown)\0", f.read())
    return m.group(1).decode() if m else None


def stale(path=LIB):
    return lib_build_id(path) != source_digest()


def build(force=False, verbose=False, out=LIB):
    """Compile the library to `out` (in-tree by default) unless it already
    carries the sources' build id."""
    if not force and not stale(out):
        return out
    bid = source_digest()
    odir = os.path.dirname(os.path.abspath(out))
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(odir, os.path.basename(src) + ".o")
        cmd = [hipcc(), "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
               "-I" + os.path.join(ROOT, "include"), f'-DZC_BUILD_ID="{bid}"', "-c", src, "-o", obj]
        if os.path.basename(src) in HOST_ONLY:
            cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-Wall", "-I" + os.path.join(ROOT, "include"),
                   "-c", src, "-o", obj]
        elif src.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd), cmd))  # the sources compile in parallel
        objs.append(obj)
    failed = [(p.returncode, cmd) for p, cmd in procs if p.wait() != 0]
    if failed:
        for o in objs:
            if os.path.exists(o):
                os.remove(o)
        raise subprocess.CalledProcessError(*failed[0])
    tmp = out + ".tmp"
    cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs
    subprocess.run(cmd, check=True)
    for o in objs:
        os.remove(o)
    os.replace(tmp, out)  # a failed build never leaves a half-written library
    if lib_build_id(out) != bid:
        raise RuntimeError(f"{out}: build id missing after the build")
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
