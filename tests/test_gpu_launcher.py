"""``python -m chanamq_amd.server --data-plane gpu`` as a product: configured from a HOCON
file (chana.mq.gpu.* tables, store dir, flow watermarks, AMQPS keystore), a TLS client
publishes persistent messages with confirms, the server is killed and restarted from the
same config, and the messages come back (AMQPServer.scala:52-106)."""

import os
import signal
import socket
import subprocess
import sys
import time

import pytest

from chanamq_amd.client import Connection

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _wait_port(port, proc, timeout=120):
    end = time.time() + timeout
    while time.time() < end:
        if proc.poll() is not None:
            raise AssertionError(f"server exited with {proc.returncode}")
        try:
            socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
            return
        except OSError:
            time.sleep(0.2)
    raise AssertionError("server did not come up")


def _start(conf, log):
    env = dict(os.environ, PYTHONPATH=ROOT)
    return subprocess.Popen([sys.executable, "-m", "chanamq_amd.server", "--config", str(conf), "--stats-interval", "1"],
                            cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT)


def test_gpu_server_from_config_tls_store_restart(gpu, tmp_path):
    from test_tls import make_cert
    key, crt, _ = make_cert(tmp_path)
    port, tport, aport = _free_port(), _free_port(), _free_port()
    conf = tmp_path / "gpu.conf"
    conf.write_text(f"""
chana.mq.amqp.server {{ interface = "127.0.0.1", port = {port} }}
chana.mq.amqps.server {{ interface = "127.0.0.1", port = {tport}, enable = true }}
chana.mq.ssl {{ cert = "{crt}", key = "{key}" }}
chana.mq.amqp.admin.port = {aport}
chana.mq.amqp.connection.heartbeat = 0
chana.mq.store {{ dir = "{tmp_path / 'store'}", fsync = true }}
chana.mq.flow {{ memory-high-watermark = 48000000, memory-low-watermark = 24000000 }}
chana.mq.gpu {{
  enable = true, io-threads = 2, max-connections = 64, channels-per-connection = 8, max-queues = 64,
  max-exchanges = 64, max-consumers = 256, max-segments-per-step = 64, max-commands-per-step = 4096,
  max-deliveries-per-step = 4096, message-table = 16384, body-log-bytes = 67108864, queue-ring-pool = 1048576,
  queue-capacity = 4096, unacked-window = 256, ingress-bytes = 8388608, egress-bytes = 16777216,
  carry-bytes = 262144, topic-bindings = 64, persist-records = 4096, persist-bytes = 8388608
}}
""")
    log1 = open(tmp_path / "s1.log", "w")
    p1 = _start(conf, log1)
    try:
        _wait_port(tport, p1)
        c = Connection(port=tport, tls=True)
        ch = c.channel()
        ch.exchange_declare("cfg.x", "direct", durable=True)
        ch.queue_declare("cfg.q", durable=True)
        ch.queue_bind("cfg.q", "cfg.x", "k")
        ch.confirm_select()
        for i in range(20):
            ch.basic_publish("cfg.x", "k", b"durable-%d" % i, {"delivery_mode": 2})
        assert ch.wait_for_confirms()
        import json
        import urllib.request
        st = json.loads(urllib.request.urlopen(f"http://127.0.0.1:{aport}/admin/stats").read())
        assert st["connections_open"] >= 1
        c.close()
    finally:
        p1.send_signal(signal.SIGTERM)
        p1.wait(timeout=60)
    log2 = open(tmp_path / "s2.log", "w")
    p2 = _start(conf, log2)
    try:
        _wait_port(port, p2)
        c2 = Connection(port=port)
        ch2 = c2.channel()
        ch2.basic_consume("cfg.q", "back", no_ack=True)
        got = ch2.consume_n(20)
        assert [g.body for g in got] == [b"durable-%d" % i for i in range(20)]
        c2.close()
    finally:
        p2.send_signal(signal.SIGTERM)
        p2.wait(timeout=60)
    assert "recovered 20 messages" in open(tmp_path / "s2.log").read()


@pytest.mark.timeout(300)
def test_gpu_server_default_sizing_carries_a_12mb_message(gpu, tmp_path):
    """The shipped chana.mq.gpu defaults (64 GiB body log, 16 M message table, 16 MiB
    largest message) come up on one MI355X, and a 12 MB message goes through the device
    path intact."""
    port = _free_port()
    conf = tmp_path / "default.conf"
    conf.write_text(f"""
chana.mq.amqp.server {{ interface = "127.0.0.1", port = {port} }}
chana.mq.amqp.admin.port = {_free_port()}
chana.mq.amqp.connection.heartbeat = 0
chana.mq.gpu.enable = true
""")
    with open(tmp_path / "srv.log", "w") as log:
        p = _start(conf, log)
        try:
            _wait_port(port, p)
            c = Connection(port=port, vhost="/")
            ch = c.channel()
            ch.queue_declare("big")
            body = os.urandom(12 << 20)
            ch.basic_publish("", "big", body)
            cc = c.channel()
            cc.basic_consume("big", "bc", no_ack=True)
            got = cc.consume_n(1, timeout=60)[0]
            assert got.body == body
            c.close()
        finally:
            p.send_signal(signal.SIGTERM)
            p.wait(60)
