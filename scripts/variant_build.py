"""Timing-only variant of libdal.so: one source file of csrc/ compiled from a
patched copy in /tmp (every `OLD=>NEW` pair given in a patch file must match
once), linked with the product build's other objects into ab/NAME/libdal.so.
The product source is not modified.
usage: python scripts/variant_build.py NAME SOURCE.hip PATCHFILE ["-DDAL_X=1 ..."]
PATCHFILE: blocks separated by a line '=====', each OLD, a line '-----', NEW
(or '-': no patch); the optional last argument adds compile flags (tuning
constants) for the patched source."""
import glob
import os
import subprocess
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
CSRC = os.path.join(REPO, "distributed-active-learning_amd", "csrc")
name, src_name, patch = sys.argv[1:4]
extra = sys.argv[4].split() if len(sys.argv) > 4 else []
s = open(os.path.join(CSRC, src_name)).read()
for block in [] if patch == "-" else open(patch).read().split("\n=====\n"):
    old, new = block.split("\n-----\n")
    assert s.count(old) == 1, old[:80]
    s = s.replace(old, new)
out = os.path.join(REPO, "ab", name)
os.makedirs(out, exist_ok=True)
# a private directory: a stray common.hpp beside the copy would shadow csrc's
# (the quoted include searches the copy's own directory first)
os.makedirs(f"/tmp/dal_variant_{name}", exist_ok=True)
tmp = f"/tmp/dal_variant_{name}/{src_name}"
open(tmp, "w").write(s)
obj = os.path.join(out, src_name.replace(".hip", ".o"))
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                "-I" + os.path.join(REPO, "include"), "-I" + CSRC] + extra + ["-c", tmp, "-o", obj], check=True)
objs = [o for o in glob.glob(os.path.join(REPO, "build", "csrc", "*.o"))
        if os.path.basename(o) != os.path.basename(obj)]
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                os.path.join(out, "libdal.so")] + objs + [obj], check=True)
print("built", os.path.join(out, "libdal.so"))
