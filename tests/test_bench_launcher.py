"""bench.py's self-launch of N ranks (``--gpus N`` with no outside launcher):
a stub worker stands in for the GPU bench, so the rank environment, the
stdout routing (rank 0's headline last), and the exit-code propagation run on
the CPU.  Reference parallelism being replaced: the RDD row partitions and the
range-partition sort of density_weighting.py:47,62,73."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import textwrap

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = textwrap.dedent('''
    import json, os, sys, time
    r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["LOCAL_RANK"] == str(r)
    assert os.environ["MASTER_ADDR"] == "127.0.0.1" and int(os.environ["MASTER_PORT"]) > 0
    print(json.dumps({"extra": "cfg", "rank": r}), flush=True)
    if r == int(os.environ.get("STUB_FAIL_RANK", "-1")):
        sys.exit(3)
    if r == int(os.environ.get("STUB_HANG_RANK", "-1")):
        time.sleep(600)
    time.sleep(0.05 * (w - r))  # rank 0 ends last: other ranks' lines come first
    if r == 0:
        print(json.dumps({"metric": "m", "value": 1.0, "world_size": w}), flush=True)
''')


def _run(n, tmp_path, **env):
    stub = tmp_path / "stub.py"
    stub.write_text(STUB)
    drv = (f"import sys; sys.path.insert(0, {REPO!r}); import bench; "
           f"sys.exit(bench.launch_ranks({n}, [sys.executable, {str(stub)!r}]))")
    e = dict(os.environ, **{k: str(v) for k, v in env.items()})
    e.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, "-c", drv], env=e, capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("n", [2, 8])
def test_launcher_headline_last(n, tmp_path):
    p = _run(n, tmp_path)
    assert p.returncode == 0, p.stderr
    out = [json.loads(x) for x in p.stdout.splitlines() if x.strip()]
    # only rank 0's lines reach stdout, its headline last
    assert out[-1] == {"metric": "m", "value": 1.0, "world_size": n}
    assert [o.get("rank") for o in out[:-1]] == [0]
    # every other rank ran (its stdout went to stderr)
    err_ranks = sorted(json.loads(x)["rank"] for x in p.stderr.splitlines() if x.startswith("{"))
    assert err_ranks == list(range(1, n))


@pytest.mark.parametrize("n,fail", [(2, 1), (8, 5), (8, 0)])
def test_launcher_propagates_failure(n, fail, tmp_path):
    # the failing rank's code comes back; a rank left waiting is stopped
    p = _run(n, tmp_path, STUB_FAIL_RANK=fail, STUB_HANG_RANK=(fail + 1) % n)
    assert p.returncode == 3, (p.returncode, p.stderr)
    assert f"rank {fail} exited with 3" in p.stderr
    assert '"metric"' not in p.stdout


def test_bench_self_launch_reaches_ranks_before_gpu(tmp_path):
    """``bench.py --gpus 2`` with no WORLD_SIZE starts two ranks itself (the
    parent never imports torch); here, without a GPU, the ranks fail and the
    parent exits nonzero after naming the failing rank."""
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e["DAL_BENCH_BACKEND"] = "gloo"
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--config", "2",
                        "--out", ""], env=e, capture_output=True, text=True, timeout=300)
    if p.returncode == 0:  # (a GPU host: the gloo rehearsal ran to the end)
        assert json.loads(p.stdout.splitlines()[-1])["world_size"] == 2
        return
    assert "bench launcher: rank" in p.stderr
    assert "--gpus 2 but" not in p.stderr  # no refusal for a missing outside launcher
