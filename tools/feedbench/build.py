"""BENCH TOOLING: compile tools/feedbench/feed_bench.cpp (the zutils.cc read loop over
integration/gpu_backup_creator.hh, with a bundle-appending Writer) against libzchunk.so."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
BIN = os.path.join(HERE, "feed_bench")


def build(out=BIN):
    cmd = ["g++", "-std=c++14", "-O2", "-Wall", "-Werror", "-pthread",
           "-I" + HERE, "-I" + os.path.join(ROOT, "tests", "adapter", "mock"), "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "integration"), os.path.join(HERE, "feed_bench.cpp"),
           "-o", out, "-L" + os.path.join(ROOT, "zbackup_amd"), "-lzchunk",
           "-Wl,-rpath," + os.path.join(ROOT, "zbackup_amd"), "-Wl,-rpath,$ORIGIN/../../zbackup_amd",
           "-L/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib"]
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    print(build())
