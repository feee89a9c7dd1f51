"""Host-side pieces of bench.py (no GPU): the benchmarked pool is the
BASELINE.md pool (numpy default_rng(0)), and any row shard generated alone
(PCG64 advance) equals the same rows of the full pool, so every GPU count
benchmarks the pool the parity tests prove bit-exact."""
import numpy as np
import pytest

import bench
from oracle import dal_oracle as O


@pytest.mark.parametrize("n,d", [(300_000, 64), (70_000, 30), (140_000, 256)])
def test_host_pool_is_the_oracle_pool(n, d):
    full = O.synthetic_pool(n, d, seed=0)
    assert np.array_equal(bench.host_pool(0, n, d, "uniform"), full)
    for lo, hi in [(512, 66_560), (65_536 + 512, n), (n - 1024, n)]:
        assert np.array_equal(bench.host_pool(lo, hi, d, "uniform"), full[lo:hi])


def test_host_pool_normal_is_the_oracle_pool():
    n, d = 20_000, 30
    full = O.synthetic_pool(n, d, seed=0, dist="normal")
    assert np.array_equal(bench.host_pool(0, n, d, "normal"), full)
    assert np.array_equal(bench.host_pool(1024, 5120, d, "normal"), full[1024:5120])


def test_shard_ranges_cover_the_pool():
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(bench.__file__), "distributed-active-learning_amd"))
    from dal import parallel

    for n in (2_000_000, 284_807, 100_000):
        for world in (1, 2, 4, 8):
            got = [parallel.shard_range(n, world, r)[:2] for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
            assert all(lo % 512 == 0 for lo, _ in got)


def test_density_accuracy_host_reference():
    """bench.py's accuracy block: the host fp64 column sum and sampled-row
    densities equal a brute-force full Gram row-sum (E excluded), sharded or not."""
    rng = np.random.default_rng(5)
    x = rng.random((300, 7), dtype=np.float32)
    u = x.astype(np.float64) / np.linalg.norm(x.astype(np.float64), axis=1, keepdims=True)
    S = u @ u.T
    n_ex = 10
    d_full = S[:, n_ex:].sum(axis=1)
    s = bench.host_colsum64(x, 0, n_ex, chunk=64)
    s2 = bench.host_colsum64(x[:130], 0, n_ex, chunk=50) + bench.host_colsum64(x[130:], 130, n_ex)
    assert np.allclose(s, s2, rtol=1e-14, atol=0)
    for lo, hi in ((0, 300), (0, 130), (130, 300), (5, 12)):
        got = {}

        def dens(pick, lo=lo):
            got["pick"] = pick
            return d_full[lo + pick] * (1 + 1e-9)

        mx, mean, dmin, amax, m = bench.density_accuracy(x[lo:hi], lo, dens, s, n_ex, m=50)
        pick = got["pick"]
        assert m == len(pick) and len(pick) <= 50
        assert np.all(lo + pick >= n_ex) and pick.max() == hi - lo - 1
        assert abs(mx - 1e-9) < 1e-12 and abs(mean - 1e-9) < 1e-12
        assert np.isclose(dmin, np.abs(d_full[lo + pick]).min())
    assert bench.sample_rows(5, 0, 10, 50).size == 0


def test_abs_rowsum_tolerance():
    rng = np.random.default_rng(6)
    x = rng.standard_normal((500, 5), dtype=np.float32)
    u = x.astype(np.float64) / np.linalg.norm(x.astype(np.float64), axis=1, keepdims=True)
    S = u @ u.T
    d_full, a_full = S[:, 10:].sum(axis=1), np.abs(S[:, 10:]).sum(axis=1)
    pick = bench.sample_rows(500, 0, 10, 100)
    sub = pick[np.linspace(0, pick.size - 1, 20).round().astype(np.int64)]
    got = bench.abs_rowsum_tolerance(x, pick, lambda p: d_full[p] + 1e-7 * a_full[p], 10, m=20, chunk=64)
    assert abs(got - 1e-7) < 1e-12
    assert sub.size == 20


def test_cpu_baseline_small_pool():
    """Both CPU-baseline variants (full fp64 Gram row-sum; separable density) run on a small pool."""
    cfg = dict(bench.CONFIGS["2"])
    x = bench.host_pool(0, 3000, 16, "uniform")
    of = O.synthetic_forest(cfg["trees"], cfg["depth"], 16, seed=1, dist="uniform")
    r = bench.cpu_baseline(x, cfg, of, budget_s=0.3)
    assert r["value"] > 0 and r["kind"] == "port" and r["cores"] >= 1
    assert r["separable"]["value"] > 0 and "separable" not in r["sample"]


def test_config_specs_and_default_extras():
    """The default config-4 run also measures configs 2, 3, 5 and config 4 at
    T = 100 and k = 1000."""
    assert bench.DEFAULT_EXTRA.split(",") == ["2", "3", "5", "4:T100", "4:k1000"]
    c, cfg, label = bench.resolve("4:T100")
    assert c == "4" and cfg["trees"] == 100 and cfg["k"] == 100 and label == "config4_T100"
    c, cfg, label = bench.resolve("4:k1000")
    assert cfg["trees"] == 10 and cfg["k"] == 1000 and label == "config4_k1000"
    assert bench.CONFIGS["4"]["trees"] == 10 and bench.CONFIGS["4"]["k"] == 100  # not mutated
    assert bench.resolve("3")[2] == "config3" and bench.resolve("5")[1]["mode"] == "div"


def test_gram_roofline_frac_is_algorithmic():
    """roofline.frac = algorithmic flops / time / the 2.5 PF dense fp16 peak;
    the executed MFMA rate (3 products, symmetric pairs once) is separate."""
    r = bench.gram_roofline("sym", 1125.0, None, 1819.0, 1819.0, 2.048e15, products=3)
    assert r["peak"] == 2500.0 and abs(r["frac"] - 0.45) < 1e-12
    assert abs(r["mfma_util_executed"] - 0.675) < 1e-12
    r2 = bench.gram_roofline("sym", 1600.0, None, 1.0, 1.0, 1.0, products=2)
    assert abs(r2["mfma_util_executed"] - r2["frac"]) < 1e-12


def test_div_self_check_canonical_numpy():
    """bench's config-5 host check: numpy canonical max-cos equals the oracle's."""
    rng = np.random.default_rng(3)
    X = rng.random((300, 16))
    got = bench.canon_maxcos(X[50:], X[:20])
    ref, _ = O.max_cosine_canonical(X, np.arange(20))
    assert np.array_equal(got, ref[50:])


def _canned_result():
    """The full result of a real default run (round 3, config 4 + extras)."""
    import json
    import os

    path = os.path.join(os.path.dirname(bench.__file__), "profiles", "r03", "final_s3", "bench_line.json")
    with open(path) as f:
        out = json.load(f)
    out.update(world_size=1, backend=None)
    return out


def test_headline_is_compact_and_complete():
    """The driver keeps an ~8 KB stdout tail: the LAST line (the headline)
    must stay <= 4,000 bytes and carry the contract's keys, roofline and
    cpu_baseline (the 25 KB line was unparseable)."""
    import json

    out = _canned_result()
    out["roofline"]["kernel"] = "x" * 500  # long free text is cut, not carried
    out["cpu_baseline"]["sample"] = "y" * 2000
    h = bench.headline(out)
    s = json.dumps(h)
    assert len(s.encode()) <= bench.HEADLINE_MAX_BYTES
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config",
                "warm_selection_latency_ms", "self_check", "roofline", "roofline_forest", "roofline_topk",
                "cpu_baseline", "world_size", "backend"):
        assert key in h, key
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel"):
        assert key in h["roofline"], key
    assert len(h["roofline"]["kernel"]) <= 80
    assert set(h["cpu_baseline"]) == {"value", "unit", "cores", "kind", "sample"}
    assert all(isinstance(v, bool) for v in h["self_check"].values())
    assert h["value"] == round(out["value"], -1) or abs(h["value"] / out["value"] - 1) < 1e-5
    # a multi-GPU record names its rank count and the per-rank exchange maxima
    out.update(world_size=8, backend="nccl", n_gpus=8, sharded_path=True,
               ranks={"gram_ms_max": 160.1, "gram_ms_min": 158.0, "all_gather_ms_max": 3.2})
    h8 = bench.headline(out)
    assert h8["world_size"] == 8 and h8["backend"] == "nccl" and h8["ranks"]["all_gather_ms_max"] == 3.2
    assert h8["sharded_path"] is True
    assert len(json.dumps(h8).encode()) <= bench.HEADLINE_MAX_BYTES


def test_emit_prints_extras_then_headline_last(tmp_path, capsys):
    import json

    out = _canned_result()
    bench.emit(out, str(tmp_path / "full.json"))
    lines = capsys.readouterr().out.strip().split("\n")
    assert len(lines) == len(out["extra"]) + 1
    for line, label in zip(lines, out["extra"]):
        e = json.loads(line)
        assert e["extra"] == label and len(line.encode()) <= bench.EXTRA_MAX_BYTES
    last = json.loads(lines[-1])
    assert last["metric"] == bench.METRIC and "roofline" in last and "cpu_baseline" in last
    assert len(lines[-1].encode()) <= bench.HEADLINE_MAX_BYTES
    full = json.load(open(tmp_path / "full.json"))  # every sub-field kept in the file
    assert full["roofline"]["kernel_note"] if "kernel_note" in full["roofline"] else full["roofline"]["kernel"]
    assert set(full["extra"]) == set(out["extra"])
