"""The sharded front end on the CPU (csrc/core/frontend.cpp stepper_sharded): two rank
processes, each an EchoEngine(world=2) behind its own Frontend, stepping in lockstep over
the real shared-memory exchange (csrc/kernels/xchg_host.h).  Covered: cross-rank records
imported one step later, the busy flag, a control-sync request on one rank parking every
rank at the same step, and failover when a peer dies mid-run (bounded exchange wait ->
FE_XFAIL -> rebuilt exchange over the survivor)."""

import os
import re
import socket
import subprocess
import sys
import time
import uuid

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _read_until(s, token, timeout=10.0):
    s.settimeout(0.2)
    buf = b""
    end = time.time() + timeout
    while token not in buf and time.time() < end:
        try:
            chunk = s.recv(65536)
        except socket.timeout:
            continue
        if not chunk:
            break
        buf += chunk
    assert token in buf, (token, buf[-200:])
    return buf


def _start(tmp_path, world, mode):
    name = "cmq-test-" + uuid.uuid4().hex[:12]
    procs, ports = [], []
    for r in range(world):
        out = str(tmp_path / f"rank{r}.port")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "frontend_sharded_worker.py"), str(r),
                                       str(world), name, out, mode], stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for r in range(world):
        out = tmp_path / f"rank{r}.port"
        end = time.time() + 60
        while not out.exists():
            assert procs[r].poll() is None, procs[r].stdout.read()
            assert time.time() < end
            time.sleep(0.05)
        ports.append(int(out.read_text()))
    return procs, ports


def _stop(tmp_path, procs):
    for r in range(len(procs)):
        (tmp_path / f"rank{r}.port.stop").write_text("")
    for p in procs:
        try:
            p.wait(20)
        except subprocess.TimeoutExpired:
            p.kill()


@pytest.fixture(params=["sync", "async"])
def ranks(tmp_path, request):
    procs, ports = _start(tmp_path, 2, request.param)
    yield procs, ports, tmp_path
    _stop(tmp_path, procs)


def _conn(port):
    s = socket.create_connection(("127.0.0.1", port))
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    return s


@pytest.mark.timeout(120)
def test_lockstep_exchange_sync_and_failover(ranks):
    procs, ports, tmp = ranks
    c0, c1 = _conn(ports[0]), _conn(ports[1])
    time.sleep(0.3)
    # echo on the local rank
    c0.sendall(b"hello0")
    assert _read_until(c0, b"hello0").endswith(b"hello0")
    # cross-rank: the bytes after XR1 travel through the exchange to rank 1's slot 1
    c0.sendall(b"abcXR1world")
    _read_until(c0, b"abc")
    _read_until(c1, b"world")
    c1.sendall(b"xyzXR0back")
    _read_until(c0, b"back")
    for i in range(50):   # a burst both ways, order kept per connection
        c0.sendall(b"XR1m%03d." % i)
    got = _read_until(c1, b"m049.")
    assert [int(x) for x in re.findall(rb"m(\d{3})\.", got)] == list(range(50))
    # a control command on rank 1: both ranks park at the same step, twice in a row (the
    # second sync is requested while the first is handled, as an owner's link_got answer)
    c1.sendall(b"CTRL")
    s1 = _read_until(c1, b";", timeout=10)
    s1 += _read_until(c1, b";") if s1.count(b";") < 2 else b""
    s0 = _read_until(c0, b";", timeout=10)
    s0 += _read_until(c0, b";") if s0.count(b";") < 2 else b""
    n1 = [int(x) for x in re.findall(rb"SYNC(\d+);", s1)]
    n0 = [int(x) for x in re.findall(rb"SYNC(\d+);", s0)]
    assert n0 == n1 and len(n0) == 2 and n0[0] > 0 and n0[1] > n0[0], (s0, s1)
    c1.sendall(b"after-sync")
    _read_until(c1, b"after-sync")
    # rank 1 dies: rank 0's next exchange times out, it fails over and serves alone
    procs[1].kill()
    procs[1].wait(10)
    c0.sendall(b"ping")
    buf = _read_until(c0, b"FAILOVER", timeout=20)
    c0.sendall(b"alone")
    _read_until(c0, b"alone")
    assert procs[0].poll() is None
    c0.close()
    c1.close()


@pytest.mark.timeout(180)
def test_eight_ranks_async_exchange_sync_and_three_killed(tmp_path):
    """Eight ranks on the asynchronous exchange (each step's exchange on the engine's
    exchange thread, phase B behind it, results one step later): records cross a ring of
    ranks, a control sync parks all eight at the same step, then ranks 2, 5 and 7 die --
    every survivor's exchange fails, it fails over and keeps serving."""
    world = 8
    procs, ports = _start(tmp_path, world, "async")
    try:
        cs = [_conn(p) for p in ports]
        time.sleep(0.3)
        for r in range(world):   # r -> r+1
            cs[r].sendall(b"r%dXR%dfrom%d." % (r, (r + 1) % world, r))
        for r in range(world):
            _read_until(cs[(r + 1) % world], b"from%d." % r)
        cs[3].sendall(b"CTRL")
        got = [_read_until(c, b";", timeout=15) for c in cs]
        steps = [re.findall(rb"SYNC(\d+);", g)[0] for g in got]
        assert len(set(steps)) == 1, steps
        for r in (2, 5, 7):
            procs[r].kill()
            procs[r].wait(10)
        live = [r for r in range(world) if r not in (2, 5, 7)]
        for r in live:
            cs[r].sendall(b"ping")
        for r in live:
            _read_until(cs[r], b"FAILOVER", timeout=30)
            cs[r].sendall(b"alone%d" % r)
            _read_until(cs[r], b"alone%d" % r)
            assert procs[r].poll() is None
        for c in cs:
            c.close()
    finally:
        _stop(tmp_path, procs)
    per_step = []
    for r in live:
        xs, xn, _, xf = (tmp_path / f"rank{r}.port.stats").read_text().split()
        per_step.append(1e6 * float(xs) / max(1, int(xn)))
        assert int(xf) >= 1
    print("stepper exchange us/step per surviving rank:", [round(v, 1) for v in per_step])
