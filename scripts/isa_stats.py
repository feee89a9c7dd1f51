"""Instruction counts of the gfx950 code objects in a libdal.so build (A/B
and ablation builds: did a change keep every MFMA? how many VALU / LDS ops?).

usage: python scripts/isa_stats.py LIB.so [LIB.so ...] [--kernel SUBSTR]"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def functions(lib):
    with tempfile.TemporaryDirectory() as tmp:
        p = os.path.join(tmp, "lib.so")
        shutil.copy(lib, p)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", p], cwd=tmp, check=True, capture_output=True)
        for f in sorted(os.listdir(tmp)):
            if "gfx950" not in f:
                continue
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", os.path.join(tmp, f)], capture_output=True,
                                 text=True).stdout
            for chunk in re.split(r"\n(?=[0-9a-f]+ <)", dis):
                m = re.match(r"[0-9a-f]+ <(.*?)>:", chunk)
                if m:
                    yield m.group(1), chunk


def stats(body):
    ins = re.findall(r"^\s+([a-z_0-9]+)", body, re.M)
    c = {"total": len(ins)}
    c["mfma"] = sum(i.startswith("v_mfma") for i in ins)
    c["valu"] = sum(i.startswith("v_") and not i.startswith("v_mfma") for i in ins)
    c["ds"] = sum(i.startswith("ds_") for i in ins)
    c["vmem"] = sum(i.startswith(("global_", "buffer_", "flat_")) for i in ins)
    c["barrier"] = sum(i == "s_barrier" for i in ins)
    c["waitcnt"] = sum(i.startswith("s_waitcnt") for i in ins)
    return c


def main():
    args = sys.argv[1:]
    sub = "gram_csym_kernel"
    if "--kernel" in args:
        i = args.index("--kernel")
        sub = args[i + 1]
        del args[i:i + 2]
    for lib in args:
        print(f"== {lib}")
        for name, body in functions(lib):
            if sub in name:
                print(f"  {name[:70]:70s} {stats(body)}")


if __name__ == "__main__":
    main()
