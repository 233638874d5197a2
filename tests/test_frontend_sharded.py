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


@pytest.fixture
def ranks(tmp_path):
    name = "cmq-test-" + uuid.uuid4().hex[:12]
    procs, ports = [], []
    for r in range(2):
        out = str(tmp_path / f"rank{r}.port")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "frontend_sharded_worker.py"), str(r), "2",
                                       name, out], stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for r in range(2):
        out = tmp_path / f"rank{r}.port"
        end = time.time() + 60
        while not out.exists():
            assert procs[r].poll() is None, procs[r].stdout.read()
            assert time.time() < end
            time.sleep(0.05)
        ports.append(int(out.read_text()))
    yield procs, ports, tmp_path
    for r in range(2):
        (tmp_path / f"rank{r}.port.stop").write_text("")
    for p in procs:
        try:
            p.wait(20)
        except subprocess.TimeoutExpired:
            p.kill()


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
