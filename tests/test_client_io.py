"""Regression tests for the test client's socket handling.

``Connection.process()`` used to end with ``_pump(0.0)``, which put the socket in
non-blocking mode; a later ``sendall`` against a peer that was not reading then raised
``BlockingIOError(11)`` (GPUTEST_r03: ``test_mixed_clients_across_ranks``).  Here a
scripted fake broker completes the handshake and then stops reading for a while, so
the client's send buffer fills right after polls with expired windows.
"""

import socket
import threading
import time

from chanamq_amd.client import Connection
from chanamq_amd.protocol.codec import CommandAssembler, FrameParser, Method, encode_method_frame


class _StallingBroker:
    """Handshake + channel.open, then sleep ``stall`` seconds, then drain forever."""

    def __init__(self, stall):
        self.stall = stall
        self.ls = socket.socket()
        self.ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.ls.bind(("127.0.0.1", 0))
        self.ls.listen(1)
        self.port = self.ls.getsockname()[1]
        self.drained = 0
        self.stop = False
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _expect(self, s, parser, asm, buf, name):
        while True:
            while buf:
                fr = buf.pop(0)
                cmd = asm.feed(fr)
                if cmd is not None and cmd.method.name == name:
                    return cmd
            data = s.recv(65536)
            if not data:
                raise EOFError
            buf.extend(parser.feed(data))

    def _run(self):
        s, _ = self.ls.accept()
        hdr = b""
        while len(hdr) < 8:
            hdr += s.recv(8 - len(hdr))
        s.sendall(encode_method_frame(0, Method("connection.start", version_major=0, version_minor=9,
                                                server_properties={"product": "fake"},
                                                mechanisms=b"PLAIN", locales=b"en_US")))
        parser, buf = FrameParser(), []
        asm0 = CommandAssembler()
        self._expect(s, parser, asm0, buf, "connection.start_ok")
        s.sendall(encode_method_frame(0, Method("connection.tune", channel_max=16, frame_max=131072,
                                                heartbeat=0)))
        self._expect(s, parser, asm0, buf, "connection.tune_ok")
        self._expect(s, parser, asm0, buf, "connection.open")
        s.sendall(encode_method_frame(0, Method("connection.open_ok", known_hosts="")))
        self._expect(s, parser, CommandAssembler(), buf, "channel.open")
        s.sendall(encode_method_frame(1, Method("channel.open_ok", channel_id=b"")))
        time.sleep(self.stall)          # not reading: the client's send buffer fills
        s.settimeout(0.5)
        while not self.stop:
            try:
                d = s.recv(1 << 20)
            except socket.timeout:
                continue
            if not d:
                break
            self.drained += len(d)
        s.close()


def test_process_then_publish_against_stalled_peer():
    fb = _StallingBroker(stall=1.0)
    c = Connection(port=fb.port, timeout=10.0)
    ch = c.channel()
    c.sock.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 65536)
    body = b"x" * 65536
    sent = 0
    t0 = time.time()
    for _ in range(256):             # 16 MB >> socket buffers: sendall must block, not raise
        c.process(0.0)               # expired window: a poll
        c.process(0.001)
        ch.basic_publish("", "q", body)
        sent += len(body)
    assert time.time() - t0 >= 0.5   # we really did block on the stalled peer
    c._pump(-1.0)                    # negative window: still a poll, never non-blocking mode
    assert c.sock.gettimeout() == 10.0
    deadline = time.time() + 10
    while fb.drained < sent and time.time() < deadline:
        time.sleep(0.05)
    fb.stop = True
    assert fb.drained >= sent
    c.sock.close()
