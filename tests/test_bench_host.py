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
