"""Build the C++/OpenMP CPU baseline (oracle/cpu/voxcpu.cpp) in-tree as
oracle/cpu/libvoxcpu.so.  Test / measurement infrastructure (oracle rules):
loaded only by bench.py's cpu_baseline leg and tests/."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "voxcpu.cpp")
LIB = os.path.join(HERE, "libvoxcpu.so")
# x86-64-v3 = AVX2 + FMA: every x86 host a GPU box here has (no AVX-512 assumed)
FLAGS = ["-O3", "-march=x86-64-v3", "--param=sra-max-scalarization-size-Ospeed=8192", "-fopenmp", "-std=c++17", "-shared", "-fPIC"]


def build(force=False):
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(SRC):
        return LIB
    subprocess.run(["g++", *FLAGS, SRC, "-o", LIB], check=True)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
