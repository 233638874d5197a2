"""Multi-process sharded node on CPU (gloo): replicated control log, lockstep steps, and
failover — a rank dies at a step boundary, the survivors agree, rebuild the communicator,
re-home its queues and keep delivering (SURVEY §3.6 / P6 exit test, non-persistent)."""

import json
import os
import subprocess
import sys
import tempfile

import pytest

from chanamq_amd.parallel.shard import ShardMap
from test_sharded_golden import _free_port

HERE = os.path.dirname(os.path.abspath(__file__))


def _run(world, die_rank=-1, die_after=-1, scen="fanout"):
    d = tempfile.mkdtemp()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world),
               PYTHONPATH=os.pathsep.join([os.path.dirname(HERE), HERE]))
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "node_worker.py"), scen, d, str(die_rank),
                               str(die_after)], env=dict(env, RANK=str(r))) for r in range(world)]
    for p in procs:
        assert p.wait(timeout=240) == 0
    out = {}
    for r in range(world):
        f = os.path.join(d, f"rank{r}.json")
        if os.path.exists(f):
            with open(f) as fh:
                out[r] = json.load(fh)
    return out


@pytest.mark.timeout(300)
def test_lockstep_fanout_three_ranks():
    out = _run(3)
    assert sorted(q for r in out.values() for q in r["owned"]) == [f"q{i}" for i in range(6)]
    for r in out.values():
        for c, n in r["deliveries"].items():
            assert n == 8 * 3 * 5, (c, n)       # every rank's publishes reach every queue


@pytest.mark.timeout(300)
def test_failover_rehomes_queues():
    out = _run(3, die_rank=2, die_after=4)
    assert set(out) == {0, 1}
    orig = ShardMap(3)
    for r, o in out.items():
        assert o["live"] == [0, 1]
        assert o["failovers"] and o["failovers"][0][0] == [2]
        for q in o["owned"]:
            c = str(100 + int(q[1:]))
            if orig.owner("AMQ.DEFAULT", q) == r:
                assert o["deliveries"][c] == 4 * 3 * 5 + 4 * 2 * 5, (r, q, o["deliveries"][c])
            else:   # re-homed from rank 2 in step 4: everything published from then on
                assert o["deliveries"][c] == 4 * 2 * 5, (r, q, o["deliveries"][c])
    assert sorted(q for o in out.values() for q in o["owned"]) == [f"q{i}" for i in range(6)]


@pytest.mark.timeout(300)
def test_failover_reloads_durable_queues():
    """HA: rank 2 dies holding persistent messages on its durable
    queues; the survivors that inherit those queues reload them from rank 2's store and
    every message any rank published is delivered exactly once."""
    out = _run(3, die_rank=2, die_after=4, scen="durable")
    assert set(out) == {0, 1}
    orig = ShardMap(3)
    total = 0
    for r, o in out.items():
        assert o["live"] == [0, 1]
        for q in o["owned"]:
            c = str(200 + int(q[1:]))
            # steps 0-3: 3 ranks x 5 persistent messages, steps 4-7: 2 ranks x 5
            assert o["deliveries"].get(c) == 4 * 3 * 5 + 4 * 2 * 5, (r, q, o["deliveries"], o["failovers"])
            total += o["deliveries"][c]
        moved_here = [q for q in o["owned"] if orig.owner("AMQ.DEFAULT", q) == 2]
        assert o["failovers"][0][2] == 4 * 3 * 5 * len(moved_here)
        assert o["rows"] == 0            # consumed (auto-ack): the store rows are gone too
    assert total == 6 * 100


@pytest.mark.timeout(300)
def test_remote_consumer_rank_dies_messages_return_to_the_queue():
    """The consumer's rank dies holding unacked deliveries of a remote queue: the owner
    closes the link, the messages go back to the queue, and a consumer on the owner gets
    every message that was published."""
    out = _run(3, die_rank=1, die_after=6, scen="links")
    assert set(out) == {0, 2}
    assert out[2]["links"] == [] and out[2]["local"]
    assert out[2]["deliveries"].get("30") == 10 * 5, out[2]


@pytest.mark.timeout(300)
def test_remote_consumer_survives_its_queue_owner_dying():
    """The queue's owner dies: the queue re-homes to a survivor, the link re-attaches
    there and the remote consumer keeps receiving new publishes."""
    out = _run(3, die_rank=2, die_after=5, scen="links")
    assert set(out) == {0, 1}
    assert out[1]["links"] == [7]
    # steps 5..9 are published after the failover (5 messages each)
    assert out[1]["deliveries"].get("20", 0) >= 5 * 5, out[1]
