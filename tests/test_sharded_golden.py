"""Sharded data plane on CPU: ShardMap properties, an in-process cluster of golden
planes vs the single-plane oracle, and a real 2-process gloo all-to-all run."""

import os
import socket
import subprocess
import sys
import tempfile
from collections import Counter

import pytest

from chanamq_amd.engine.golden import GoldenDataPlane
from chanamq_amd.parallel.cluster import LocalCluster
from chanamq_amd.parallel.shard import ShardMap
from sharded_scenarios import SHARDED, apply, split_inputs

HERE = os.path.dirname(os.path.abspath(__file__))


def golden(**kw):
    return GoldenDataPlane(default_queue_capacity=1 << 12, ring_pool=1 << 20, **kw)


def run_single(spec, world):
    """Oracle: one plane holding every connection, connection ids remapped so their
    order is (rank, connection) — the cross-rank enqueue order of the sharded plane."""
    remap = {c: (r % world) * 256 + c for c, r in spec.rank_of.items()}
    back = {v: k for k, v in remap.items()}
    dp = golden()
    apply(dp, spec, conn_map=remap)
    out = []
    for k, st in enumerate(spec.steps):
        eg = dp.step({remap[c]: b for c, b in st.items()}, now_ms=1000 + k)["egress"]
        out.append({back[c]: b for c, b in eg.items()})
    return out


def run_cluster(spec, world):
    cl = LocalCluster(lambda **kw: golden(**kw), world)
    for r in range(world):
        apply(cl[r], spec, rank=r, world=world)
    outs = []
    for k, st in enumerate(spec.steps):
        res = cl.step(split_inputs(spec, st, world), now_ms=1000 + k)
        merged = {}
        for r in res:
            for c, b in r["egress"].items():
                assert c not in merged
                merged[c] = b
        outs.append(merged)
    return outs


def test_shard_map_balance_and_minimal_movement():
    m = ShardMap(8)
    own = {i: m.owner("/", f"q{i}") for i in range(8000)}
    cnt = Counter(own.values())
    assert set(cnt) == set(range(8)) and min(cnt.values()) > 850
    m.fail(5)
    moved = [i for i in own if m.owner("/", f"q{i}") != own[i]]
    assert all(own[i] == 5 for i in moved) and len(moved) == cnt[5]
    m.place("/", "pinned", 3)
    assert m.owner("/", "pinned") == 3


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", sorted(SHARDED))
def test_cluster_matches_single_plane(name, world):
    spec = SHARDED[name]()
    single = run_single(spec, world)
    clus = run_cluster(SHARDED[name](), world)
    assert len(single) == len(clus)
    for k, (a, b) in enumerate(zip(single, clus)):
        assert set(a) == set(b), (k, sorted(a), sorted(b))
        for c in a:
            assert a[c] == b[c], (k, c)
    assert any(single), "scenario produced no egress"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name", ["topic", "fanout_confirm"])
def test_gloo_two_process_matches_single_plane(name):
    """One process per rank, gloo all_to_all_single (the RCCL code path on CPU)."""
    spec = SHARDED[name]()
    single = run_single(spec, 2)
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="2",
                   PYTHONPATH=os.pathsep.join([os.path.dirname(HERE), HERE]))
        procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "sharded_worker.py"), name, d, "golden"],
                                  env=dict(env, RANK=str(r))) for r in range(2)]
        for p in procs:
            assert p.wait(timeout=240) == 0
        import json
        got = [dict() for _ in spec.steps]
        for r in range(2):
            with open(os.path.join(d, f"rank{r}.json")) as f:
                for k, eg in enumerate(json.load(f)):
                    for c, hx in eg.items():
                        got[k][int(c)] = bytes.fromhex(hx)
    for k, (a, b) in enumerate(zip(single, got)):
        assert a == b, k


def run_cluster_lag(spec, world, extra_steps=2):
    cl = LocalCluster(lambda **kw: golden(exchange_lag=1, **kw), world)
    for r in range(world):
        apply(cl[r], spec, rank=r, world=world)
    outs = []
    for k, st in enumerate(spec.steps + [{}] * extra_steps):
        res = cl.step(split_inputs(spec, st, world), now_ms=1000 + k)
        merged = {}
        for r in res:
            merged.update(r["egress"])
        outs.append(merged)
    return outs


@pytest.mark.parametrize("world", [2, 3])
def test_lagged_exchange_delivers_the_same_messages(world):
    """exchange_lag=1 (pipelined collective): cross-rank publishes arrive one step later,
    but every consumer gets the same deliveries as the single-plane oracle (fanout)."""
    import re
    spec = SHARDED["fanout_confirm"]()
    single = run_single(spec, world)
    lag = run_cluster_lag(SHARDED["fanout_confirm"](), world)

    def bodies(outs, c):
        blob = b"".join(o.get(c, b"") for o in outs)
        return len(re.findall(rb"\x01\x00\x01\x00\x00\x00.\x00\x3c\x00\x3c", blob, re.S))
    for c in range(20, 28):
        assert bodies(single, c) == bodies(lag, c) > 0, c
