"""Sharded GPU data plane (HIP, gfx950): W ranks on one device stepped in lockstep
(LocalCluster, device-to-device exchange) and two processes exchanging over gloo, both
byte-compared with the single-plane golden oracle (tests/test_sharded_golden.py)."""

import json
import os
import subprocess
import sys
import tempfile

import pytest

from gpu_cfg import CFG
from sharded_scenarios import SHARDED, apply, split_inputs
from test_sharded_golden import _free_port, run_cluster_lag, run_single

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def run_gpu_cluster(spec, world, graph=True, lag=0, extra_steps=0, cfg=None):
    import torch

    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.parallel.cluster import LocalCluster
    torch.cuda.set_device(0)
    c = dict(CFG, **(cfg or {}))
    cl = LocalCluster(lambda **kw: GpuDataPlane(graph=graph, exchange_lag=lag, **c, **kw), world)
    for r in range(world):
        apply(cl[r], spec, rank=r, world=world)
    outs = []
    for k, st in enumerate(spec.steps + [{}] * extra_steps):
        res = cl.step(split_inputs(spec, st, world), now_ms=1000 + k)
        merged = {}
        for r in res:
            merged.update(r.egress)
        outs.append(merged)
    return outs


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", sorted(SHARDED))
def test_gpu_cluster_matches_oracle(gpu, name, world):
    single = run_single(SHARDED[name](), world)
    got = run_gpu_cluster(SHARDED[name](), world)
    for k, (a, b) in enumerate(zip(single, got)):
        assert set(a) == set(b), (k, sorted(a), sorted(b))
        for c in a:
            assert a[c] == b[c], (k, c)


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("name", sorted(SHARDED))
def test_gpu_cluster_wide_pair_keys(gpu, name, world):
    """q_max 512: pair keys of 10-11 bits (queue << rank_bits | rank), sorted in the single
    11-bit radix pass, queue starts read from its digit offsets (no k_qfirst)."""
    single = run_single(SHARDED[name](), world)
    got = run_gpu_cluster(SHARDED[name](), world, cfg=dict(q_max=512))
    for k, (a, b) in enumerate(zip(single, got)):
        assert set(a) == set(b), (k, sorted(a), sorted(b))
        for c in a:
            assert a[c] == b[c], (k, c)


def test_gpu_cluster_eager_matches_graph(gpu):
    a = run_gpu_cluster(SHARDED["topic"](), 2, graph=True)
    b = run_gpu_cluster(SHARDED["topic"](), 2, graph=False)
    assert a == b


def _two_process_gpu(spec_name, steps, lag=False):
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="2",
                   PYTHONPATH=os.pathsep.join([os.path.dirname(HERE), HERE]))
        procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "sharded_worker.py"), spec_name, d, "gpu"]
                                  + (["lag"] if lag else []), env=dict(env, RANK=str(r))) for r in range(2)]
        for p in procs:
            assert p.wait(timeout=360) == 0
        got = [dict() for _ in range(steps)]
        for r in range(2):
            with open(os.path.join(d, f"rank{r}.json")) as f:
                for k, eg in enumerate(json.load(f)):
                    for c, hx in eg.items():
                        got[k][int(c)] = bytes.fromhex(hx)
    return got


@pytest.mark.timeout(400)
def test_gpu_two_process_exchange(gpu):
    """One process per rank (both on device 0), gloo all_to_all with host staging."""
    spec = SHARDED["fanout_confirm"]()
    assert run_single(spec, 2) == _two_process_gpu("fanout_confirm", len(spec.steps))


@pytest.mark.timeout(400)
@pytest.mark.parametrize("name", ["fanout_confirm", "topic"])
def test_gpu_two_process_pipelined_exchange(gpu, name):
    """The benchmark's exchange schedule, one process per rank: step t's ingress is queued
    (deferred launch), step t-1's all-to-all runs, then step t's kernels import it --
    byte-identical to the golden cluster with exchange_lag=1."""
    want = run_cluster_lag(SHARDED[name](), 2, extra_steps=2)
    assert _two_process_gpu(name, len(want), lag=True) == want


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", sorted(SHARDED))
def test_gpu_lagged_exchange_matches_golden(gpu, name, world):
    """exchange_lag=1: the HIP cluster and the golden cluster agree byte for byte."""
    want = run_cluster_lag(SHARDED[name](), world, extra_steps=2)
    got = run_gpu_cluster(SHARDED[name](), world, lag=1, extra_steps=2)
    for k, (a, b) in enumerate(zip(want, got)):
        assert set(a) == set(b), (k, sorted(a), sorted(b))
        for c in a:
            assert a[c] == b[c], (k, c)


@pytest.mark.timeout(180)
def test_rccl_single_rank_paths(gpu):
    """RCCL on the device: the bench's all-to-all exchange (device tensors, exact splits,
    empty steps) and all_reduce through a one-rank communicator, and the engine's dlopen'ed
    librccl binding (every symbol resolved, a unique id drawn)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="1", RANK="0",
               LOCAL_RANK="0", PYTHONPATH=os.path.dirname(HERE))
    p = subprocess.run([sys.executable, os.path.join(HERE, "rccl_single_worker.py")], env=env,
                       capture_output=True, text=True, timeout=170)
    assert p.returncode == 0 and "RCCL ok" in p.stdout, (p.returncode, p.stdout[-2000:], p.stderr[-3000:])
