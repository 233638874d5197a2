"""Mixed-client soak against the GPU-data-path server: confirm-mode publishers with
mandatory unroutable publishes, a manual-ack consumer settling with every Ack / Nack /
Reject combination (single, multiple, both kinds back to back in one step), an auto-ack
consumer that cancels and re-consumes, and a Basic.Get client that rejects and recovers,
all at once.  Invariants: every routable publish is settled-as-consumed exactly once,
every unroutable one comes back as a Basic.Return, all confirms are acks and the plane
holds nothing afterwards.  (The settle-order bug this round — an Ack(multiple) applied
before an earlier Nack(multiple, requeue) of the same step — breaks "exactly once".)"""

import os
import random
import threading
import time

import pytest

from chanamq_amd.client import Connection
from test_gpu_broker import GPU_CFG, SMALL, _gpu_present

SMALL_CONF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sharded_small.conf")

N_PUB, PER_PUB, QUEUES = 2, 500, 4


def make_plane(kind, persist=False):
    if kind == "golden":
        from chanamq_amd.engine.golden import GoldenDataPlane
        return GoldenDataPlane(default_queue_capacity=1 << 12, ring_pool=1 << 20, persist=persist, **SMALL)
    if not _gpu_present():
        pytest.fail("GPU test scheduled on a machine without a GPU")
    from chanamq_amd.engine.dataplane import GpuDataPlane
    return GpuDataPlane(default_queue_capacity=1 << 12, persist=int(persist), **GPU_CFG)


@pytest.fixture(params=["golden-native", pytest.param("gpu-pipeline", marks=pytest.mark.gpu),
                        pytest.param("gpu-native", marks=pytest.mark.gpu), "golden-native-store",
                        pytest.param("gpu-pipeline-store", marks=pytest.mark.gpu)])
def broker(request, tmp_path):
    from chanamq_amd.broker import load
    from chanamq_amd.server.gpu_broker import GpuBroker
    kind, io, *store = request.param.split("-")
    st = None
    if store:   # durable queues, persistent messages, the WAL store behind them
        st = load().Store()
        st.open(str(tmp_path / "store"), False)
    b = GpuBroker(make_plane(kind, persist=bool(store)), idle_step_ms=1.0, io=io, ingress_bytes=8 << 20,
                  store=st).start()
    b.durable = bool(store)
    b.store_handle = st
    yield b
    b.stop()
    if st is not None:
        st.close()


class Soak:
    def __init__(self, port, ports=None, durable=False):
        self.port, self.durable = port, durable
        self.ports = ports or {}   # client role -> port (sharded: a rank per role)
        self.lock = threading.Lock()
        self.done = []            # bodies settled as consumed (ack / auto-ack)
        self.routable, self.unroutable, self.returned = set(), set(), []
        self.nacked_confirms = 0
        self.pubs_left = N_PUB
        self.errors = []

    def conn(self, role=""):
        return Connection(port=self.ports.get(role, self.port), vhost="/")

    def finished(self):
        with self.lock:
            return self.pubs_left == 0 and len(self.done) >= len(self.routable)

    def _consumed(self, bodies):
        with self.lock:
            self.done.extend(bodies)

    # ------------------------------------------------------------------ clients
    def publisher(self, pid):
        rng = random.Random(pid)
        c = self.conn("pub%d" % pid)
        ch = c.channel()
        ch.confirm_select()
        mine_r, mine_u = set(), set()
        for i in range(PER_PUB):
            body = b"p%d-%d" % (pid, i)
            props = {"delivery_mode": 2} if self.durable else None
            if rng.random() < 0.05:
                ch.basic_publish("sx", "nokey", body, props, mandatory=True)
                mine_u.add(body)
            else:
                ch.basic_publish("sx", "k%d" % rng.randrange(QUEUES), body, props)
                mine_r.add(body)
            if i % 25 == 24:
                c.process(0.002)
        with self.lock:
            self.routable |= mine_r
            self.unroutable |= mine_u
        ok = ch.wait_for_confirms(timeout=30)
        c.process(0.2)
        with self.lock:
            self.returned += [d.body for d in ch.returns]
            self.nacked_confirms += 0 if ok else 1
            self.pubs_left -= 1
        c.close()

    def mixer(self, deadline):
        """q0 + q1 on one channel (prefetch 30), every settle pattern."""
        rng = random.Random(7)
        c = self.conn("mixer")
        ch = c.channel()
        ch.basic_qos(prefetch_count=30)
        ch.basic_consume("q0", "m0")
        ch.basic_consume("q1", "m1")
        out = {}   # tag -> body (unsettled)
        while time.time() < deadline and not self.finished():
            c.process(0.01)
            while ch.deliveries:
                d = ch.deliveries.popleft()
                out[d.method.delivery_tag] = d.body
            if not out:
                continue
            tags = sorted(out)
            r = rng.random()
            if r < 0.35:     # ack everything (multiple)
                ch.basic_ack(tags[-1], multiple=True)
                self._consumed([out.pop(t) for t in tags])
            elif r < 0.6:    # nack the first half (requeue), then ack the rest, back to back
                mid = tags[len(tags) // 2]
                ch.basic_nack(mid, multiple=True, requeue=True)
                ch.basic_ack(tags[-1], multiple=True)
                self._consumed([out.pop(t) for t in tags if t > mid])
                for t in tags:
                    out.pop(t, None)
            elif r < 0.85:   # one by one: ack or reject(requeue)
                acked = []
                for t in tags:
                    if rng.random() < 0.6:
                        ch.basic_ack(t)
                        acked.append(out.pop(t))
                    else:
                        ch.basic_reject(t, requeue=True)
                        out.pop(t)
                self._consumed(acked)
            else:            # nack everything (requeue)
                ch.basic_nack(tags[-1], multiple=True, requeue=True)
                out.clear()
        c.close()

    def auto(self, deadline):
        """q2, auto-ack, cancels and re-consumes every ~40 deliveries."""
        c = self.conn("auto")
        ch = c.channel()
        k, n = 0, 0
        ch.basic_consume("q2", "a0", no_ack=True)
        while time.time() < deadline and not self.finished():
            c.process(0.01)
            got = []
            while ch.deliveries:
                got.append(ch.deliveries.popleft().body)
            self._consumed(got)
            n += len(got)
            if n >= 40:
                ch.basic_cancel("a%d" % k)
                c.process(0.01)
                self._consumed([d.body for d in ch.deliveries])   # in flight before CancelOk
                ch.deliveries.clear()
                k += 1
                n = 0
                ch.basic_consume("q2", "a%d" % k, no_ack=True)
        c.close()

    def getter(self, deadline):
        """q3 by Basic.Get: ack, reject(requeue), or hold and Basic.Recover."""
        rng = random.Random(3)
        c = self.conn("getter")
        ch = c.channel()
        held = 0
        while time.time() < deadline and not self.finished():
            d = ch.basic_get("q3")
            if d is None:
                if held:
                    ch.basic_recover(requeue=True)
                    held = 0
                time.sleep(0.005)
                continue
            r = rng.random()
            if r < 0.6:
                ch.basic_ack(d.method.delivery_tag)
                self._consumed([d.body])
            elif r < 0.8:
                ch.basic_reject(d.method.delivery_tag, requeue=True)
            else:
                held += 1
                if held >= 5:
                    ch.basic_recover(requeue=True)
                    held = 0
        c.close()


def run_soak(s):
    deadline = time.time() + 90
    ths = [threading.Thread(target=fn, args=a) for fn, a in
           [(s.publisher, (p,)) for p in range(N_PUB)] + [(s.mixer, (deadline,)), (s.auto, (deadline,)),
                                                         (s.getter, (deadline,))]]

    def guard(t):
        run = t.run

        def wrapped():
            try:
                run()
            except Exception as e:   # surfaced below
                s.errors.append(repr(e))
        t.run = wrapped
        return t
    for t in ths:
        guard(t).start()
    for t in ths:
        t.join(120)
    print("soak:", len(s.done), "consumed,", len(s.returned), "returned,", len(s.routable), "routable")
    assert not s.errors, s.errors
    assert s.nacked_confirms == 0
    assert sorted(s.returned) == sorted(s.unroutable)
    assert len(s.done) == len(set(s.done)), "a message was consumed twice"
    assert set(s.done) == s.routable


def _topology(port, queues, durable=False):
    c = Connection(port=port, vhost="/")
    ch = c.channel()
    ch.exchange_declare("sx", "direct", durable=durable)
    for q in queues:
        ch.queue_declare("q%d" % q, durable=durable)
        ch.queue_bind("q%d" % q, "sx", "k%d" % q)
    c.close()


@pytest.mark.timeout(180)
def test_mixed_clients_every_message_consumed_exactly_once(broker):
    _topology(broker.port, range(QUEUES), broker.durable)
    run_soak(Soak(broker.port, durable=broker.durable))
    time.sleep(0.3)
    with broker.lock:
        assert broker.plane.memory_in_use() == 0
    if broker.durable:   # the store agrees: every persistent message's rows are gone
        time.sleep(0.3)
        with broker.lock:
            if broker.persistence.native is not None:
                broker.persistence.native.drain()
            st = broker.store_handle
            left = {q: (len(r[1]), len(r[2])) for q in st.queue_ids() if (r := st.select_queue(q)) and (r[1] or r[2])}
            assert not left, left
            assert not st.message_ids()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("plane", ["golden", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_mixed_clients_across_ranks(tmp_path, plane):
    """Two ranks of the sharded server (gloo): q0/q1 live on rank 0 and are
    consumed by the mixer on rank 1 (links), q2/q3 live on rank 1 and are consumed on rank
    0 by the auto-ack consumer (link) and the Basic.Get client (get link); a publisher on
    each rank."""
    import json
    import os

    from chanamq_amd.parallel.launch import Launcher
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, PYTHONPATH=os.path.dirname(here))
    extra = ["--backend", "gloo"] if plane == "gpu" else []   # 2 ranks share the one test GPU
    ln = Launcher(2, ["-m", "chanamq_amd.server.sharded", "--config", SMALL_CONF, "--plane", plane, "--port", "0",
                      "--info-dir", str(tmp_path)] + extra, env=env).start()
    try:
        deadline = time.time() + 120
        while time.time() < deadline and not all((tmp_path / f"rank{r}.json").exists() for r in range(2)):
            assert not ln.poll(), f"rank exited early: {ln.poll()}"
            time.sleep(0.2)
        ports = [json.load(open(tmp_path / f"rank{r}.json"))["port"] for r in range(2)]
        _topology(ports[0], (0, 1))
        _topology(ports[1], (2, 3))
        s = Soak(ports[0], ports=dict(pub0=ports[0], pub1=ports[1], mixer=ports[1], auto=ports[0],
                                      getter=ports[0]))
        run_soak(s)
    finally:
        ln.stop()
