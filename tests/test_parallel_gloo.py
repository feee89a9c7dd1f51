"""Multi-process orchestration of dal.parallel over gloo (CPU, world_size 2,
3, 4 and 8).  The two exchanges (all-gather of normalised shards + canonical column
sum partials, all-gather of local top-k) and the deterministic merge are the
product code; the per-shard arithmetic (HIP on the GPU) is replaced here by the
oracle, so the test covers sharding, collectives and merge order on CPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dal import parallel
from dal.luts import lut
from oracle import dal_oracle as O

N, D, K = 2600, 12, 50


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class OracleShard(parallel.ShardedSelector):
    """ShardedSelector with the per-shard steps computed by the oracle (CPU)."""

    def __init__(self, X, n_total, rank, world, excluded, of):
        self.n_total, self.rank, self.world = n_total, rank, world
        self.lo, self.hi, self.shard = parallel.shard_range(n_total, world, rank)
        self.x = X[self.lo:self.hi]
        self.excluded = np.asarray(excluded)
        self.of = of
        self._density = None
        self._parts_full = None

    def prep(self):
        ex = O.exclusion_mask(self.n_total, self.excluded)[self.lo:self.hi]
        u = torch.zeros((self.shard, D), dtype=torch.float64)
        parts = torch.zeros((self.shard // 256, D), dtype=torch.float64)
        if self.hi > self.lo:
            U = O.l2_normalize(self.x)
            U[ex] = 0.0
            u[: U.shape[0]] = torch.from_numpy(U)
            for c in range((U.shape[0] + 255) // 256):
                acc = np.zeros(D)
                for r in range(c * 256, min(U.shape[0], c * 256 + 256)):
                    if not ex[r]:
                        acc = acc + U[r]
                parts[c] = torch.from_numpy(acc)
        return u, parts

    def exchange_density(self, comm, u_local, parts=None):
        return comm.all_gather(u_local), (comm.all_gather(parts) if parts is not None else None)

    def index_tensor(self, unl):
        return torch.as_tensor(np.asarray(unl), dtype=torch.int64)

    def status_word(self):
        # a forced re-rank capacity overflow on one rank's first attempt: every
        # rank must see it (OR of the gathered words) and redo the step
        if getattr(self, "overflow_once", False) and not getattr(self, "retries", 0):
            from dal import _lib

            return torch.full((1,), _lib.DAL_FLAG_CAND_OVERFLOW, dtype=torch.int32)
        return torch.zeros(1, dtype=torch.int32)

    def prepare_retry(self, sample_miss=False):
        self.retries = getattr(self, "retries", 0) + 1

    def local_select(self, u_full, parts_full, unl, forest, k, mode="dw", strategy="least_confidence",
                     beta=1.0, density_mode="gram", warm=None):
        keys = torch.full((k,), parallel._as_i64(0xFFFFFFFFFFFFFFFF), dtype=torch.int64)
        idx = torch.full((k,), -1, dtype=torch.int64)
        sc = torch.full((k,), float("nan"), dtype=torch.float64)
        unl = np.asarray(unl)
        mine = unl[(unl >= self.lo) & (unl < self.hi)]
        if mine.size == 0:
            return parallel.LocalTopk(keys, idx, sc)
        s = np.zeros(D)
        for c in range(parts_full.shape[0]):
            s = s + parts_full[c].numpy()
        U = O.l2_normalize(self.x[mine - self.lo])
        dd = np.zeros(mine.size)
        for f in range(D):
            dd = dd + U[:, f] * s[f]
        dd[np.isin(mine, self.excluded)] = np.nan
        v = O.votes(self.of, self.x[mine - self.lo])
        score = lut("entropy", self.of.n_trees)[v] * dd
        si, ss = O.select_topk(score, mine, k, ascending=False)
        kk = si.size
        keys[:kk] = torch.from_numpy(_float_key(ss))
        idx[:kk] = torch.from_numpy(si)
        sc[:kk] = torch.from_numpy(ss)
        return parallel.LocalTopk(keys, idx, sc)


def _float_key(s):
    """Test-side mirror of score_key (descending, NaN last, -0 == +0)."""
    s = np.where(s == 0, 0.0, s)
    b = s.view(np.uint64)
    u = np.where(b >> np.uint64(63), ~b, b | np.uint64(1 << 63))
    k = ~u
    k = np.where(np.isnan(s), np.uint64(0xFFFFFFFFFFFFFFFE), k)
    return k.view(np.int64)


def _cpu_sort_positions(keys, pos, k):
    u = keys.numpy().view(np.uint64)
    order = np.lexsort((pos.numpy(), u))[:k]
    return torch.from_numpy(order.astype(np.int64))


def _worker(rank, world, port, q, case="all"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _run(rank, world, q, case)
    except Exception as e:  # surface worker failures instead of a queue timeout
        q.put((rank, repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


def _unlabeled(case):
    """The unlabeled set of a case: every row outside L0, or with holes --
    all of rows [512, 1024) labeled (at world >= 4 one rank has no unlabeled
    row at all) and a scatter of labeled rows elsewhere."""
    unl = np.arange(10, N)
    if case != "all":
        unl = unl[(unl < 512) | (unl >= 1024)]
        unl = unl[unl % 7 != 3]
    return unl


def _run(rank, world, q, case):
    X = O.synthetic_pool(N, D, seed=4)
    of = O.synthetic_forest(10, 4, D, seed=1)
    E = np.arange(10)
    sel = OracleShard(X, N, rank, world, E, of)
    sel.overflow_once = case == "retry" and rank == world - 2
    idx, sc = parallel.select(sel, parallel.TorchComm(), _unlabeled(case), None, K, mode="dw",
                              sort_fn=_cpu_sort_positions)
    q.put((rank, idx.numpy(), sc.numpy(), getattr(sel, "retries", 0)))


@pytest.mark.parametrize("world,case", [(2, "all"), (3, "all"), (4, "holes"), (8, "holes"), (8, "retry")])
def test_gloo_sharded_density_select_matches_oracle(world, case):
    """World 4 / 8 shards are uneven (N = 2600: 512-row shards, the last
    non-empty one holds 40 rows -- fewer than k -- and at world 8 two ranks
    hold none); "holes": one rank's rows are all labeled; "retry": one rank
    reports a re-rank capacity overflow and every rank redoes the step."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, case)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    X = O.synthetic_pool(N, D, seed=4)
    of = O.synthetic_forest(10, 4, D, seed=1)
    _, ref_idx, ref_sc = O.density_select(X, _unlabeled(case), of, K, 1.0, np.arange(10))
    for rank, idx, sc, retries in res:
        assert not isinstance(idx, str), idx
        assert np.array_equal(idx, ref_idx), rank
        assert np.array_equal(sc, ref_sc), rank
        assert retries == (1 if case == "retry" else 0), (rank, retries)


def test_shard_ranges_cover_pool():
    for n in (1, 511, 512, 100_000, 2_000_000, 284_807):
        for w in (1, 2, 3, 4, 8):
            rows = []
            for r in range(w):
                lo, hi, s = parallel.shard_range(n, w, r)
                assert s % 512 == 0 and hi - lo <= s
                rows.append((lo, hi))
            assert rows[0][0] == 0 and rows[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rows, rows[1:]))


def test_other_column_ranges_cover_the_rest():
    for world in (1, 2, 3, 8):
        shard = 1024
        for rank in range(world):
            cols = set()
            for c0, c1 in parallel.other_column_ranges(rank, world, shard):
                assert c0 % 512 == 0 and c1 % 512 == 0 and c0 < c1
                cols.update(range(c0, c1))
            own = set(range(rank * shard, (rank + 1) * shard))
            assert cols.isdisjoint(own) and cols | own == set(range(world * shard))


def _comm_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = parallel.TorchComm()
        # fp16-split Gram operands travel as uint16 bit patterns (no gloo type)
        u = (torch.arange(6, dtype=torch.int32) + 1000 * rank + 60000).to(torch.uint16).view(3, 2)
        g = comm.all_gather(u)
        # the warm step's packed top-k row (int64)
        row = torch.arange(7, dtype=torch.int64) + 100 * rank
        rows = comm.all_gather_rows(row)
        q.put((rank, g.dtype == torch.uint16, g.to(torch.int32).numpy(), rows.numpy()))
    except Exception as e:
        q.put((rank, repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


def test_gloo_comm_unsigned_gather_and_rows():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_g = np.concatenate([np.arange(6).reshape(3, 2) + 1000 * r + 60000 for r in range(world)])
    want_rows = np.stack([np.arange(7) + 100 * r for r in range(world)])
    for rank, is_u16, g, rows in res:
        assert is_u16 is True, is_u16
        assert np.array_equal(g, want_g)
        assert np.array_equal(rows, want_rows)
