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


def _standin_env():
    from chanamq_amd import ops
    so = ops.build_rccl_standin()
    assert so and os.path.exists(so), "tests/rccl_standin/librccl_standin.so not built"
    return {"CHANAMQ_RCCL_LIB": so, "CHANAMQ_RCCL_STANDIN_OK": "1"}


def _native_procs(spec_name, world, kind, steps, extra=()):
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world),
                   PYTHONPATH=os.pathsep.join([os.path.dirname(HERE), HERE]), **_standin_env())
        procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "native_xchg_worker.py"), spec_name, d, kind]
                                  + list(extra), env=dict(env, RANK=str(r))) for r in range(world)]
        for p in procs:
            assert p.wait(timeout=300) == 0
        got = [dict() for _ in range(steps)]
        for r in range(world):
            with open(os.path.join(d, f"rank{r}.json")) as f:
                for k, eg in enumerate(json.load(f)):
                    for c, hx in eg.items():
                        got[k][int(c)] = bytes.fromhex(hx)
    return got


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world,name,extra", [(2, "topic", ()), (2, "fanout_confirm", ("counts_shm",)),
                                              (3, "direct_manual_ack", ()), (4, "fanout_confirm", ())])
def test_engine_rccl_exchange_multi_rank_matches_golden(gpu, world, name, extra):
    """The engine's RCCL exchange (xchg_rccl.h RcclXchg: count exchange and bulk as grouped
    ncclSend / ncclRecv, bounded event waits) with 2-4 ranks, one process each, all on the
    one test GPU through the tests' librccl stand-in (real RCCL refuses two ranks on one
    device): byte-identical to the golden cluster with the pipelined exchange."""
    want = run_cluster_lag(SHARDED[name](), world, extra_steps=2)
    got = _native_procs(name, world, "rccl", len(want), extra)
    for k, (a, b) in enumerate(zip(want, got)):
        assert set(a) == set(b), (k, sorted(a), sorted(b))
        for c in a:
            assert a[c] == b[c], (k, c)


_MISMATCH = r'''
import ctypes, os, sys
L = ctypes.CDLL(os.environ["CHANAMQ_RCCL_LIB"])
rank, uid_hex = int(sys.argv[1]), sys.argv[2]
class Uid(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]
uid = Uid.from_buffer_copy(bytes.fromhex(uid_hex))
comm = ctypes.c_void_p()
assert L.ncclCommInitRank(ctypes.byref(comm), 2, uid, rank) == 0
bufs = [ctypes.create_string_buffer(512) for _ in range(4)]
def group(ops):
    L.ncclGroupStart()
    bad = 0
    for send, i, n in ops:
        f = L.ncclSend if send else L.ncclRecv
        bad |= f(bufs[i], ctypes.c_size_t(n), 0, 1 - rank, comm, None)
    return L.ncclGroupEnd() or bad
ctypes.memmove(bufs[0], b"x" * 100, 100)
# a matched group first: both sides agree
r1 = group([(True, 0, 100), (False, 1, 100)])
# then the receiver posts its second part one byte longer than the sender sent
r2 = group([(True, 0, 100), (True, 2, 200)] if rank == 0 else [(False, 1, 100), (False, 3, 201)])
print("RESULT", rank, r1, r2, flush=True)
L.ncclCommDestroy(comm)
'''


@pytest.mark.timeout(120)
def test_rccl_standin_fails_loudly_on_mismatched_parts(gpu):
    """The stand-in is stricter than NCCL: a peer's group whose part sizes differ from the
    receives this rank posted fails the group (ncclInvalidUsage) and aborts the
    communicator, so an exchange whose two sides disagree cannot pass a test."""
    env = dict(os.environ, **_standin_env())
    uid = (b"CMQSTND\0" + f"/cmq-rccl-standin-mm-{os.getpid()}".encode()).ljust(128, b"\0").hex()
    procs = [subprocess.Popen([sys.executable, "-c", _MISMATCH, str(r), uid], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=100) for p in procs]
    res = {}
    for out, err in outs:
        for line in out.splitlines():
            if line.startswith("RESULT"):
                _, r, r1, r2 = line.split()
                res[int(r)] = (int(r1), int(r2))
    assert res.get(0, (None,))[0] == 0 and res.get(1, (None,))[0] == 0, (res, outs)
    assert res[1][1] == 5, (res, outs)            # ncclInvalidUsage on the receiving side
    assert "mismatch" in outs[1][1], outs[1][1][-500:]
