"""The REAL RCCL branch of the sharded selection, on one GPU.

A spawned child initialises ``torch.distributed`` with the ``nccl`` backend
(RCCL on ROCm) at world size 1 on cuda:0 and drives ``dal.parallel`` through
the real ``TorchComm``.  RCCL refuses two ranks on one device, so world size 1
is the largest RCCL group one GPU can hold; at world size 1 every collective
is still a real RCCL call on the communicator's stream, so this exercises the
code that only runs under RCCL (gloo stages through the host instead):

* ``TorchComm.overlaps``: the own-shard Gram queued first on the reduced grid,
  then the operand and partials all-gathered asynchronously from a side
  stream, ``record_stream`` + ``wait`` on the main stream
  (``ShardedSelector.exchange_density``), with and without the exchange's
  timing events;
* the uint16 split operand moved as bytes (``TorchComm.all_gather_start``);
* the warm step: ``ShardedSelector.warm_plan`` replay whose packed row goes
  through ``TorchComm.all_gather_rows`` into the kept buffer, then the
  one-launch ``dal_topk_merge`` (two warm steps: the second reuses the plan
  and the buffer);
* uncertainty sampling and the sharded diversity selection.

Indices and fp64 score bits must equal the CPU oracle's, and the sharded
results must equal the single-GPU engine's bit for bit.

Reference: density_weighting.py:73 (BlockMatrix shuffle), :168,:172 (sortBy +
take to the driver); uncertainty_sampling.py:106,109; similarity.py:34-38.
"""
import os
import socket

import numpy as np
import pytest

from oracle import dal_oracle as O

pytestmark = pytest.mark.gpu

N, D, K = 6000, 64, 50
N2, D2 = 3000, 256  # a second pool: the KS-128 operand, a 256-wide byte view


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _np(t):
    return t.detach().cpu().numpy()


def _worker(port, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (repo, os.path.join(repo, "distributed-active-learning_amd"), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from dal import engine, parallel
        from dal.forest import Forest

        comm = parallel.TorchComm()
        out = {"backend": comm.backend, "overlaps": bool(comm.overlaps), "world": comm.world}
        X = O.synthetic_pool(N, D, seed=33)
        F = Forest.synthetic(10, 4, D, seed=1)
        E = np.arange(10)
        unl = np.arange(10, N)
        x = torch.from_numpy(X).to(dev)

        sel = parallel.ShardedSelector(x, N, 0, 1, excluded=E, device=dev)
        u_local, _ = sel.prep()
        out["operand_dtype"] = str(u_local.dtype)
        out["operand_needs_bytes"] = bool(parallel._needs_bytes(u_local.dtype))
        # cold step with the exchange's timing events (side-stream event branch)
        sel.exchange_events = []
        idx, sc = parallel.select(sel, comm, unl, F, K, mode="dw")
        torch.cuda.synchronize()
        out["ag_events"] = [(nm, float(a.elapsed_time(b))) for nm, a, b in sel.exchange_events]
        sel.exchange_events = None
        out["dw_cold_events"] = (_np(idx), _np(sc))
        # cold step without events (the product's branch)
        sel.clear_caches()
        idx, sc = parallel.select(sel, comm, unl, F, K, mode="dw")
        out["dw_cold"] = (_np(idx), _np(sc))
        out["dens_bits"] = _np(sel.state.density("gram").view(torch.int64))
        # two warm steps: plan replay -> all_gather_rows -> one-launch merge
        idx, sc = parallel.select(sel, comm, unl, F, K, mode="dw")
        out["dw_warm1"] = (_np(idx), _np(sc))
        idx, sc = parallel.select(sel, comm, unl, F, K, mode="dw")
        out["dw_warm2"] = (_np(idx), _np(sc))
        out["n_plans"] = len(sel._plans)
        out["rows_buffers"] = len(comm._rows)
        # a different unlabeled set on the warm path (later-labeled rows drop out)
        unl2 = np.setdiff1d(unl, out["dw_warm2"][0])
        idx, sc = parallel.select(sel, comm, unl2, F, K, mode="dw")
        out["dw_warm_unl2"] = (_np(idx), _np(sc))
        # the single-GPU engine on the same pool: the same bits
        st = engine.PoolState(x, excluded=E, device=dev)
        r = engine.density_step(st, torch.from_numpy(unl).to(dev), F, K)
        out["single"] = (_np(r.indices), _np(r.selected_scores))
        out["single_dens_bits"] = _np(st.density("gram").view(torch.int64))

        # uncertainty sampling (no normalisation; a zero row is legal)
        X0 = X.copy()
        X0[77] = 0.0
        sel_us = parallel.ShardedSelector(torch.from_numpy(X0).to(dev), N, 0, 1, device=dev)
        for strat in ("least_confidence", "margin", "entropy"):
            idx, sc = parallel.select(sel_us, comm, np.arange(N), F, K, mode="us", strategy=strat)
            out["us_" + strat] = (_np(idx), _np(sc))

        # a 256-wide pool (KS-128 operand) at k = 100: cold, then warm
        X2 = O.synthetic_pool(N2, D2, seed=34)
        F2 = Forest.synthetic(10, 4, D2, seed=2)
        sel2 = parallel.ShardedSelector(torch.from_numpy(X2).to(dev), N2, 0, 1, excluded=E, device=dev)
        unl_b = np.arange(10, N2)
        idx, sc = parallel.select(sel2, comm, unl_b, F2, 100, mode="dw")
        out["dw256_cold"] = (_np(idx), _np(sc))
        idx, sc = parallel.select(sel2, comm, unl_b, F2, 100, mode="dw")
        out["dw256_warm"] = (_np(idx), _np(sc))

        # sharded diversity selection (bf16 pool, replicated labeled rows)
        xb = torch.from_numpy(O.bf16_round(X)).to(dev)
        lab = torch.from_numpy(O.bf16_round(X[:128])).to(dev)
        cand = np.arange(128, N)
        idx, sc = parallel.diversity_select_sharded(xb, 0, lab, 40, comm, candidates=cand, device=dev)
        out["div"] = (_np(idx), _np(sc))
        torch.cuda.synchronize()
        q.put(out)
    except Exception:  # surface worker failures instead of a queue timeout
        import traceback

        q.put(traceback.format_exc())
        raise
    finally:
        dist.destroy_process_group()


def _same(a, b):
    return np.array_equal(a[0], b[0]) and np.array_equal(np.asarray(a[1]).view(np.int64),
                                                         np.asarray(b[1]).view(np.int64))


def test_rccl_world1_sharded_paths_bit_exact(cuda):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=240)
    p.join(timeout=60)
    assert isinstance(out, dict), out
    assert p.exitcode == 0
    # the RCCL branch really ran
    assert out["backend"] == "nccl" and out["overlaps"] and out["world"] == 1
    assert out["operand_needs_bytes"], out["operand_dtype"]
    assert [nm for nm, _ in out["ag_events"]] == ["all_gather"] and out["ag_events"][0][1] >= 0
    assert out["n_plans"] == 1 and out["rows_buffers"] == 1

    X = O.synthetic_pool(N, D, seed=33)
    of = O.synthetic_forest(10, 4, D, seed=1)
    unl = np.arange(10, N)
    _, dw_idx, dw_sc = O.density_select(X, unl, of, K, 1.0, np.arange(10))
    ref = (dw_idx, dw_sc)
    for key in ("dw_cold_events", "dw_cold", "dw_warm1", "dw_warm2", "single"):
        assert _same(out[key], ref), key
    assert np.array_equal(out["dens_bits"], out["single_dens_bits"])
    unl2 = np.setdiff1d(unl, dw_idx)
    _, i2, s2 = O.density_select(X, unl2, of, K, 1.0, np.arange(10))
    assert _same(out["dw_warm_unl2"], (i2, s2))

    X0 = X.copy()
    X0[77] = 0.0
    for strat in ("least_confidence", "margin", "entropy"):
        _, ui, us = O.uncertainty_select(X0, np.arange(N), of, K, strategy=strat)
        assert _same(out["us_" + strat], (ui, us)), strat

    X2 = O.synthetic_pool(N2, D2, seed=34)
    of2 = O.synthetic_forest(10, 4, D2, seed=2)
    _, i3, s3 = O.density_select(X2, np.arange(10, N2), of2, 100, 1.0, np.arange(10))
    assert _same(out["dw256_cold"], (i3, s3)) and _same(out["dw256_warm"], (i3, s3))

    div_idx, div_sc = O.diversity_select_canonical(O.bf16_round(X), np.arange(128), 40,
                                                   candidates=np.arange(128, N))
    assert _same(out["div"], (div_idx, div_sc))
