"""AMQPS (TLS) listener: PEM cert/key and PKCS12 keystore (AMQPServer.scala:70-92)."""

import shutil
import subprocess

import pytest

from chanamq_amd.broker import load
from chanamq_amd.client import Connection

pytestmark = pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI needed to mint a test cert")


def make_cert(tmp_path):
    key, crt, p12 = tmp_path / "k.pem", tmp_path / "c.pem", tmp_path / "s.p12"
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(key), "-out", str(crt),
                    "-days", "1", "-subj", "/CN=localhost"], check=True, capture_output=True)
    subprocess.run(["openssl", "pkcs12", "-export", "-inkey", str(key), "-in", str(crt), "-out", str(p12),
                    "-passout", "pass:abcdef"], check=True, capture_output=True)
    return key, crt, p12


@pytest.mark.parametrize("kind", ["pem", "p12"])
def test_tls_publish_consume(tmp_path, kind):
    key, crt, p12 = make_cert(tmp_path)
    cfg = {"port": 0, "host": "127.0.0.1", "heartbeat": 0, "tls_enable": True, "tls_port": 0}
    if kind == "pem":
        cfg.update(tls_cert=str(crt), tls_key=str(key))
    else:
        cfg.update(tls_p12=str(p12), tls_p12_password="abcdef")
    b = load().Broker(cfg)
    b.start()
    try:
        c = Connection(port=b.tls_port, tls=True)
        ch = c.channel()
        ch.queue_declare("secure")
        body = b"z" * 300000
        ch.basic_publish("", "secure", body)
        ch.basic_consume("secure", "c", no_ack=True)
        assert ch.consume_n(1)[0].body == body
        c.close()
    finally:
        b.stop()


@pytest.mark.parametrize("kind", ["pem", "p12"])
def test_tls_proxy_terminates_for_a_plain_broker(tmp_path, kind):
    """The AMQPS front of the GPU-path server (csrc/core/tls_proxy.cpp): TLS clients on one
    port, plain AMQP to the broker's listener.  Upstream here is the host broker."""
    key, crt, p12 = make_cert(tmp_path)
    core = load()
    b = core.Broker({"port": 0, "host": "127.0.0.1", "heartbeat": 0})
    b.start()
    cfg = {"port": 0, "upstream_port": b.port}
    if kind == "pem":
        cfg.update(cert=str(crt), key=str(key))
    else:
        cfg.update(p12=str(p12), p12_password="abcdef")
    px = core.TlsProxy(cfg)
    px.start()
    try:
        conns = [Connection(port=px.port, tls=True) for _ in range(3)]
        ch = conns[0].channel()
        ch.queue_declare("via.proxy")
        body = bytes(range(256)) * 3000
        for i in range(5):
            ch.basic_publish("", "via.proxy", body + bytes([i]))
        cc = conns[1].channel()
        cc.basic_consume("via.proxy", "pc", no_ack=True)
        got = cc.consume_n(5)
        assert [g.body for g in got] == [body + bytes([i]) for i in range(5)]
        assert px.connections() == 3
        for c in conns:
            c.close()
    finally:
        px.stop()
        b.stop()
