"""Timing-only variant builds of libdal.so whose split operand keeps only the
top M significant bits of the low term L (M = 0: L = 0), to measure whether
fewer toggling operand bits let the MFMA-bound Gram hold a higher clock.
The product source is not modified (instrumented copies compiled from /tmp).
usage: python scripts/gram_lbits_build.py M [M ...]  -> ab/lbits_M/libdal.so"""
import glob
import os
import subprocess
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
CSRC = os.path.join(REPO, "distributed-active-learning_amd", "csrc")
base = open(os.path.join(CSRC, "gram_split.hip")).read()
old = "      l[e] = static_cast<_Float16>(sv - static_cast<float>(he));\n    }\n    uint16_t* dst = out + row"
assert old in base
for m in (int(a) for a in sys.argv[1:]):
    if m == 0:
        rnd = "      l[e] = static_cast<_Float16>(0.0f);\n"
    else:
        drop = 24 - m
        rnd = ("      { const unsigned b = __float_as_uint(sv - static_cast<float>(he));\n"
               f"        const float r = __uint_as_float((b + (1u << {drop - 1})) & ~((1u << {drop}) - 1u));\n"
               "        l[e] = static_cast<_Float16>(r); }\n")
    s = base.replace(old, rnd + "    }\n    uint16_t* dst = out + row")
    out = os.path.join(REPO, "ab", f"lbits_{m}")
    os.makedirs(out, exist_ok=True)
    os.makedirs(f"/tmp/dal_lbits_{m}", exist_ok=True)  # private: no stray common.hpp beside the copy
    src = f"/tmp/dal_lbits_{m}/gram_split.hip"
    open(src, "w").write(s)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                    "-I" + os.path.join(REPO, "include"), "-I" + CSRC, "-c", src, "-o",
                    os.path.join(out, "gram_split.o")], check=True)
    objs = [o for o in glob.glob(os.path.join(REPO, "build", "csrc", "*.o")) if not o.endswith("gram_split.o")]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    os.path.join(out, "libdal.so")] + objs + [os.path.join(out, "gram_split.o")], check=True)
    print("built", out)
