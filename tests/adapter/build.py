"""TEST INFRASTRUCTURE: compile tests/adapter/adapter_main.cpp (the zutils.cc
loops over integration/gpu_backup_creator.hh) against include/zchunk.h and
the stand-in zbackup types of tests/adapter/mock, linked to libzchunk.so."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
BIN = os.path.join(HERE, "adapter_main")


def build_sidecar_reader(out=os.path.join(HERE, "sidecar_read")):
    """tests/adapter/sidecar_read.cpp: the adapter's chunk-metadata file reader alone."""
    cmd = ["g++", "-std=c++11", "-O2", "-Wall", "-Werror",
           "-I" + os.path.join(HERE, "mock"), "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "integration"), os.path.join(HERE, "sidecar_read.cpp"),
           "-o", out, "-L" + os.path.join(ROOT, "zbackup_amd"), "-lzchunk",
           "-Wl,-rpath," + os.path.join(ROOT, "zbackup_amd"), "-L/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib"]
    subprocess.run(cmd, check=True)
    return out


def build(out=BIN):
    cmd = ["g++", "-std=c++11", "-O2", "-Wall", "-Werror",
           "-I" + os.path.join(HERE, "mock"), "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "integration"), os.path.join(HERE, "adapter_main.cpp"),
           "-o", out, "-L" + os.path.join(ROOT, "zbackup_amd"), "-lzchunk",
           "-Wl,-rpath," + os.path.join(ROOT, "zbackup_amd"), "-Wl,-rpath,$ORIGIN/../../zbackup_amd",
           "-L/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib"]
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    print(build())
