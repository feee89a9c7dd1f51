"""Pin the round-1 race fix in the emitted gfx950 ISA (no GPU needed).

The symmetric Gram kernel (gram_csym_kernel, csrc/gram_sym.hip) flushes
LDS fp64 row/column partials that other waves add with no-return ds_add_f64.
hipcc once emitted no lgkmcnt wait at a loop-top __syncthreads, and another
wave's flush read a column partial before the add landed (a lost partial,
seen once at 500k x 256).  The fix puts `s_waitcnt vmcnt(0) lgkmcnt(0)` in
front of every barrier; this test disassembles libdal.so's gfx950 code object
and asserts that, for every s_barrier of every gram_csym_kernel instance (and
of the max-cosine kernels, which use the same LDS-DMA ring pattern), the
nearest preceding wait on the LDS counter is lgkmcnt(0) and no LDS
instruction sits between it and the barrier.  A compiler change that drops
the wait fails here instead of silently re-opening the race.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "distributed-active-learning_amd", "dal", "libdal.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def _disassemble():
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not found")
    if not os.path.exists(LIB):
        pytest.fail("libdal.so not built (run __graft_entry__.build())")
    with tempfile.TemporaryDirectory() as tmp:
        # --offloading writes the bundles next to its input: work on a copy
        shutil.copy(LIB, os.path.join(tmp, "libdal.so"))
        subprocess.run([OBJDUMP, "--offloading", "libdal.so"], cwd=tmp, check=True, capture_output=True)
        text = []
        for f in sorted(os.listdir(tmp)):
            if f.endswith("gfx950"):
                out = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", os.path.join(tmp, f)],
                                     check=True, capture_output=True, text=True).stdout
                text.append(out)
    return "\n".join(text)


def _functions(asm):
    funcs, name, body = {}, None, []
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            if name:
                funcs[name] = body
            name, body = m.group(1), []
        elif name:
            ins = line.strip().split("//")[0].strip()
            if ins:
                body.append(ins)
    if name:
        funcs[name] = body
    return funcs


def _check(body):
    bad, n = [], 0
    for i, ins in enumerate(body):
        if not ins.startswith("s_barrier"):
            continue
        n += 1
        ok = False
        for j in range(i - 1, -1, -1):
            prev = body[j]
            if prev.startswith("ds_") or prev.startswith("buffer_") and " lds" in prev:
                break
            if prev.startswith("s_waitcnt") and "lgkmcnt(0)" in prev:
                ok = True
                break
            if prev.startswith("s_waitcnt") and "lgkmcnt" in prev:
                break
        if not ok:
            bad.append((i, body[max(0, i - 6):i + 1]))
    return n, bad


def test_every_gram_barrier_waits_for_lds():
    funcs = _functions(_disassemble())
    grams = {k: v for k, v in funcs.items() if "gram_csym_kernel" in k}
    # <KS, waves>: 32/64/128 with 4 waves, 128 with 8 (two super blocks per block)
    assert len(grams) == 4, "gram_csym_kernel<32|64|128, 4> / <128, 8> not found in libdal.so"
    for name, body in grams.items():
        n, bad = _check(body)
        assert n > 0, name
        assert not bad, (name, bad[:3])


def test_every_maxcos_barrier_waits_for_lds():
    funcs = _functions(_disassemble())
    ks = {k: v for k, v in funcs.items() if "maxcos_kernel" in k}
    assert ks
    for name, body in ks.items():
        n, bad = _check(body)
        assert n > 0, name
        assert not bad, (name, bad[:3])
