"""Host AddressSanitizer + UBSan run of the pool-ingest parser (SURVEY §5;
csrc/ingest.hip, replacing uncertainty_sampling.py:37-42 /
density_weighting.py:45-53,59-65).

scripts/asan/build.sh compiles the parser's host code with
``-fsanitize=address,undefined`` together with a driver that repeats
dal/ingest.py's chunked loader (exact-size heap buffer: a read past a chunk
or the file's last byte hits ASan's redzone).  Every case of test_ingest.py's
CPU set runs through it -- ragged rows, malformed fields, digit-group
underscores, hex / nan(chars) tokens, fp64-then-fp32 rounding, take(n),
multithreaded chunks -- plus NUL bytes, CRLF, a missing final newline, blank
files and over-long tokens; results must equal the reference's parsing
(test_ingest._ref_parse) and the sanitizers must report nothing.
``DAL_ASAN_LOG_DIR`` keeps every run's sanitizer output (profiles/r05/asan/).
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import load_golden
from test_ingest import _ref_parse, _write

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, "scripts", "asan", "build.sh")
DRIVER = os.path.join(REPO, "build", "asan", "ingest_asan_driver")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0:exitcode=86",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module")
def driver():
    if not shutil.which(os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")):
        pytest.skip("hipcc not available")
    srcs = [os.path.join(REPO, "distributed-active-learning_amd", "csrc", "ingest.hip"),
            os.path.join(REPO, "scripts", "asan", "ingest_asan_driver.cpp"), BUILD]
    if not os.path.exists(DRIVER) or os.path.getmtime(DRIVER) < max(os.path.getmtime(s) for s in srcs):
        subprocess.run(["bash", BUILD, DRIVER], check=True, capture_output=True, timeout=600)
    return DRIVER


_RUNS = [0]


def run(driver, tmp_path, path, n_samples=None, label_map=0, threads=8, chunk=64 << 20):
    ox, oy = str(tmp_path / "x.bin"), str(tmp_path / "y.bin")
    p = subprocess.run([driver, str(path), str(-1 if n_samples is None else n_samples), str(label_map),
                        str(threads), str(chunk), ox, oy], env=ENV, capture_output=True, text=True, timeout=300)
    log_dir = os.environ.get("DAL_ASAN_LOG_DIR")
    if log_dir:
        os.makedirs(log_dir, exist_ok=True)
        _RUNS[0] += 1
        with open(os.path.join(log_dir, "driver_runs.log"), "a") as fh:
            fh.write(f"--- run {_RUNS[0]}: {os.path.basename(str(path))} n={n_samples} map={label_map} "
                     f"threads={threads} chunk={chunk} exit={p.returncode}\n{p.stdout}{p.stderr}")
    assert p.returncode == 0, p.stderr[-4000:]
    assert "AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-4000:]
    kv = dict(t.split("=") for t in p.stdout.split())
    rc, rows, cols = int(kv["rc"]), int(kv["rows"]), int(kv["cols"])
    if rc:
        return rc, None, None
    X = np.fromfile(ox, dtype=np.float32).reshape(rows, cols - 1)
    y = np.fromfile(oy, dtype=np.int64)
    return 0, X, y


def same(got, ref):
    assert np.array_equal(got[0].view(np.int32), ref[0].view(np.int32))
    assert np.array_equal(got[1], ref[1])


def test_asan_fixture_and_take(driver, tmp_path):
    g = load_golden("checkerboard2x2.npz")
    p = _write(tmp_path, "cb.txt", g["X"].astype(np.float64), g["y"])
    rc, X, y = run(driver, tmp_path, p, label_map=1)
    assert rc == 0
    same((X, y), _ref_parse(p, label_map="as_is"))
    rng = np.random.default_rng(4)
    Xs = rng.standard_normal((5000, 17)) * 10.0 ** rng.integers(-8, 8, size=(5000, 17))
    p = _write(tmp_path, "s.txt", Xs, rng.choice([-1, 1], size=5000), fmt="%.17g", sep="\t")
    for n in (None, 1, 4321):
        rc, X, y = run(driver, tmp_path, p, n_samples=n)
        assert rc == 0
        same((X, y), _ref_parse(p, n_samples=n))


def test_asan_rounding_and_special_tokens(driver, tmp_path):
    vals = ["1.00000005960464477539", "1.0000000596046448", "0.1", "-3.4028235677973366e+38",
            "1e-45", "7.006492321624086e-46", "16777217", "0", "-0", "2.5e-08", "inf", "-Infinity", "NaN"]
    p = tmp_path / "r.txt"
    p.write_text("\n".join(f"{v} {v} 1" for v in vals) + "\n\n   \n")
    rc, X, y = run(driver, tmp_path, p)
    assert rc == 0
    same((X, y), _ref_parse(str(p)))


@pytest.mark.parametrize("line,ok", [
    ("1_000.5 2_5e1_0 1\n1e1_0 -0_5 1_0\n", True),
    ("1 1__0 1\n", False), ("1 _1 1\n", False), ("1 1_ 1\n", False), ("1 1_.5 1\n", False),
    ("1 1._5 1\n", False), ("1 1_e5 1\n", False), ("1 0x1p3 1\n", False), ("1 -0X10 1\n", False),
    ("1 nan(123) 1\n", False), ("1 2 x 1\n", False), ("1 2 3 1.5\n", False),
    ("1 2\x00abc 1\n", False), ("1 2 1\x00\n", False),   # embedded NUL: float() rejects it
    ("1 " + "9" * 200 + " 1\n", True),                   # longer than the stack buffer: inf, like float()
    ("1 2 " + "9" * 80 + "\n", True),                    # label beyond int64: int() reads it, maps to 1
    ("1 2 -" + "0" * 70 + "1\n", True),                  # a long -1 label
    ("1 " + "1_" * 150 + "1 1\n", True),                 # a long token with digit groups
    ("1 2 " + "1" * 70 + "x\n", False),
    ("1 2 1\r\n3 4 -1\r\n", True),                       # CRLF: '\r' is whitespace
    ("1 2 1\n3 4 -1", True),                              # no final newline
])
def test_asan_tokens(driver, tmp_path, line, ok):
    p = tmp_path / "t.txt"
    p.write_bytes(line.encode("latin-1"))
    rc, X, y = run(driver, tmp_path, p)
    if ok:
        assert rc == 0
        same((X, y), _ref_parse(str(p)))
    else:
        assert rc != 0
        with pytest.raises(ValueError):
            _ref_parse(str(p))


@pytest.mark.parametrize("text", ["1 2 3 1\n4 5 1\n", "1 2 1\n\n4 5 6 1\n", "\n\n  \n", " ", "5\n"])
def test_asan_ragged_and_empty(driver, tmp_path, text):
    p = tmp_path / "bad.txt"
    p.write_text(text)
    rc, _, _ = run(driver, tmp_path, p)
    assert rc != 0


@pytest.mark.parametrize("threads,chunk", [(8, 1 << 18), (16, 1 << 16), (3, 4099), (1, 1 << 30)])
def test_asan_multithreaded_chunks(driver, tmp_path, threads, chunk):
    rng = np.random.default_rng(9)
    Xb = rng.random((60000, 12)).astype(np.float32).astype(np.float64)
    yb = rng.choice([-1, 1], size=60000)
    p = _write(tmp_path, "big.txt", Xb, yb)
    ref = _ref_parse(p)
    rc, X, y = run(driver, tmp_path, p, threads=threads, chunk=chunk)
    assert rc == 0
    same((X, y), ref)
    rc, X, y = run(driver, tmp_path, p, n_samples=33333, threads=threads, chunk=chunk)
    assert rc == 0
    same((X, y), (ref[0][:33333], ref[1][:33333]))
    # a ragged row deep inside the second thread's segment
    lines = open(p).read().split("\n")
    lines[40000] = lines[40000] + " 7"
    (tmp_path / "rag.txt").write_text("\n".join(lines))
    rc, _, _ = run(driver, tmp_path, tmp_path / "rag.txt", threads=threads, chunk=chunk)
    assert rc != 0
