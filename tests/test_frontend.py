"""Native pipelined front end (csrc/core/frontend.cpp) on the CPU: IO threads, the
stepper pipeline, pause/resume, control events and ordering, driven by EchoEngine (every
segment's bytes come back to the same connection one step later)."""

import socket
import threading
import time

import pytest

from chanamq_amd.broker import load

FE_OPEN, FE_CLOSED, FE_HOST, FE_CTRL = 1, 2, 3, 4


def _recv_exact(s, n, timeout=10.0):
    s.settimeout(timeout)
    buf = b""
    while len(buf) < n:
        chunk = s.recv(n - len(buf))
        if not chunk:
            break
        buf += chunk
    return buf


class _Events:
    def __init__(self, fe):
        self.fe, self.seen = fe, []

    def wait(self, kind, conn=None, timeout=10.0):
        end = time.time() + timeout
        while time.time() < end:
            for i, e in enumerate(self.seen):
                if e[0] == kind and (conn is None or e[1] == conn):
                    return self.seen.pop(i)
            self.seen.extend(self.fe.poll_events(50))
        raise AssertionError(f"no event {kind} for {conn}")


@pytest.fixture(params=[1, 3], ids=["io1", "io3"])
def fe(request):
    core = load()
    eng = core.EchoEngine(c_max=64, seg_max=64, ingress_cap=1 << 20, carry_cap=1 << 16)
    f = core.Frontend(eng.c_api(), {"io_threads": request.param, "idle_step_ms": 1.0, "per_conn_read": 4096})
    f.start()
    yield f, eng
    f.stop()


def _open(f, ev):
    s = socket.create_connection(("127.0.0.1", f.port))
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    conn = ev.wait(FE_OPEN)[1]
    return s, conn


def test_host_mode_then_data_echo(fe):
    f, eng = fe
    ev = _Events(f)
    s, conn = _open(f, ev)
    s.sendall(b"HELLO")
    ev.wait(FE_HOST, conn)
    got = b""
    end = time.time() + 5
    while len(got) < 5 and time.time() < end:
        got += f.take(conn)
        time.sleep(0.01)
    assert got == b"HELLO"
    f.send(conn, b"reply:")
    f.set_data_mode(conn, b"left")           # leftover handshake bytes go first
    s.sendall(b"over")
    assert _recv_exact(s, 6) == b"reply:"
    assert _recv_exact(s, 8) == b"leftover"
    payload = bytes(range(256)) * 40         # > per_conn_read: spread over several steps
    s.sendall(payload)
    assert _recv_exact(s, len(payload)) == payload
    assert f.stats()["steps"] >= 3
    s.close()
    ev.wait(FE_CLOSED, conn)
    f.close(conn)


def test_many_connections_ordered(fe):
    f, eng = fe
    ev = _Events(f)
    socks = []
    for _ in range(12):
        s, conn = _open(f, ev)
        f.set_data_mode(conn, b"")
        socks.append((s, conn))
    msgs = {conn: b"".join(b"%d:%05d;" % (conn, i) for i in range(2000)) for _, conn in socks}

    def writer(s, data):
        for k in range(0, len(data), 777):
            s.sendall(data[k:k + 777])

    ths = [threading.Thread(target=writer, args=(s, msgs[c])) for s, c in socks]
    for t in ths:
        t.start()
    for s, c in socks:
        assert _recv_exact(s, len(msgs[c])) == msgs[c]
    for t in ths:
        t.join()
    st = f.stats()
    assert st["rx_bytes"] >= sum(len(m) for m in msgs.values())
    for s, _ in socks:
        s.close()


def test_control_pause_orders_replies_after_egress(fe):
    f, eng = fe
    ev = _Events(f)
    s, conn = _open(f, ev)
    f.set_data_mode(conn, b"")
    s.sendall(b"data-before|CTRL")
    e = ev.wait(FE_CTRL, conn)
    assert e[4] == b"CTRL"
    f.pause()                                 # the step's egress ("data-before|") is out
    f.send(conn, b"<ctrl-reply>")
    eng.unpause(conn)
    f.kick(conn)
    f.resume()
    assert _recv_exact(s, len(b"data-before|<ctrl-reply>")) == b"data-before|<ctrl-reply>"
    s.sendall(b"after")
    assert _recv_exact(s, 5) == b"after"
    s.close()


def test_pause_is_exclusive_and_nests(fe):
    f, eng = fe
    ev = _Events(f)
    s, conn = _open(f, ev)
    f.set_data_mode(conn, b"")
    f.pause()
    f.pause()
    before = eng.steps
    s.sendall(b"x" * 100)
    time.sleep(0.1)
    assert eng.steps == before               # no step while paused
    f.resume()
    time.sleep(0.05)
    assert eng.steps == before
    f.resume()
    assert _recv_exact(s, 100) == b"x" * 100
    s.close()
