"""Protocol conversation tests against the native broker.

Replays the reference's manual clients (SimplePublisher / SimpleConsumer) and walks the
§2.11 method matrix, including the quirk decisions of SURVEY Appendix A.
"""

import time

import pytest

from chanamq_amd.broker import load
from chanamq_amd.client import ChannelClosed, Connection, ConnectionClosed


@pytest.fixture()
def broker(tmp_path):
    core = load()
    b = core.Broker({"port": 0, "host": "127.0.0.1", "heartbeat": 0, "data_dir": str(tmp_path / "data")})
    b.start()
    yield b
    b.stop()


def conn(b, **kw):
    return Connection(port=b.port, **kw)


def test_handshake_server_properties(broker):
    c = conn(broker)
    props = c.server_properties
    assert props["product"] in ("chana.mq", b"chana.mq")
    c.close()


def test_protocol_header_mismatch_gets_our_header(broker):
    import socket
    s = socket.create_connection(("127.0.0.1", broker.port))
    s.sendall(b"AMQP\x00\x00\x08\x00")
    s.settimeout(3)
    assert s.recv(8) == b"AMQP\x00\x00\x09\x01"
    s.close()


def test_simple_publisher_consumer_scenario(broker):
    """SimplePublisher.scala:21-54 / SimpleConsumer.scala:21,61."""
    p = conn(broker)
    ch = p.channel()
    ch.exchange_declare("test_exchange", "direct", durable=True)
    ch.queue_declare("test_queue", durable=True, arguments={"x-message-ttl": 60000})
    ch.queue_bind("test_queue", "test_exchange", "quote")
    for i in range(5):
        props = {"delivery_mode": 2} if i < 2 else {}
        if i == 1:
            props["expiration"] = "100000"
        ch.basic_publish("test_exchange", "quote", f"quote {i}".encode(), props)
    c = conn(broker)
    cc = c.channel()
    cc.basic_consume("test_queue", "myConsumerTag", no_ack=True)
    got = cc.consume_n(5)
    assert [d.body for d in got] == [f"quote {i}".encode() for i in range(5)]
    assert all(d.method.consumer_tag == "myConsumerTag" for d in got)
    p.close()
    c.close()


def test_default_exchange_and_generated_names(broker):
    c = conn(broker)
    ch = c.channel()
    ok = ch.queue_declare("")
    assert ok.queue.startswith("tmp.")
    ch.basic_publish("", ok.queue, b"x")
    tag = ch.basic_consume(ok.queue, "", no_ack=True)
    assert tag.startswith("amq.ctag-")
    d = ch.consume_n(1)[0]
    assert d.body == b"x" and d.method.exchange == ""
    c.close()


def test_topic_and_fanout_and_headers_routing(broker):
    c = conn(broker)
    ch = c.channel()
    ch.exchange_declare("t", "topic")
    ch.exchange_declare("f", "fanout")
    ch.exchange_declare("h", "headers")
    for q in ("a", "b", "c", "hq"):
        ch.queue_declare(q)
    ch.queue_bind("a", "t", "forex.*")
    ch.queue_bind("b", "t", "quote.#")
    ch.queue_bind("c", "f", "")
    ch.queue_bind("a", "f", "")
    ch.queue_bind("hq", "h", "", arguments={"x-match": "all", "k": "v"})
    ch.basic_publish("t", "forex.eur", b"1")
    ch.basic_publish("t", "quote.a.b", b"2")
    ch.basic_publish("t", "forex", b"3")
    ch.basic_publish("f", "whatever", b"4")
    ch.basic_publish("h", "", b"5", {"headers": {"k": "v"}})
    ch.basic_publish("h", "", b"6", {"headers": {"k": "w"}})
    time.sleep(0.1)
    assert ch.queue_declare("a", passive=True).message_count == 2
    assert ch.queue_declare("b", passive=True).message_count == 1
    assert ch.queue_declare("c", passive=True).message_count == 1
    assert ch.queue_declare("hq", passive=True).message_count == 1
    c.close()


def test_exchange_to_exchange_binding(broker):
    c = conn(broker)
    ch = c.channel()
    ch.exchange_declare("src", "direct")
    ch.exchange_declare("dst", "fanout")
    ch.queue_declare("e2e")
    ch.queue_bind("e2e", "dst")
    ch.exchange_bind("dst", "src", "rk")
    ch.basic_publish("src", "rk", b"via-e2e")
    time.sleep(0.05)
    assert ch.queue_declare("e2e", passive=True).message_count == 1
    c.close()


def test_mandatory_return_and_confirm_after_return(broker):
    c = conn(broker)
    ch = c.channel()
    ch.confirm_select()
    ch.basic_publish("amq.direct", "nowhere", b"lost", mandatory=True)
    assert ch.wait_for_confirms()
    c.process(0.1)
    assert len(ch.returns) == 1 and ch.returns[0].method.reply_code == 312
    c.close()


def test_immediate_without_consumers_returns_313(broker):
    c = conn(broker)
    ch = c.channel()
    ch.queue_declare("imm")
    ch.basic_publish("", "imm", b"now", immediate=True)
    c.process(0.2)
    assert ch.returns and ch.returns[0].method.reply_code == 313
    assert ch.queue_declare("imm", passive=True).message_count == 0
    c.close()


def test_prefetch_and_manual_ack(broker):
    c = conn(broker)
    ch = c.channel()
    ch.queue_declare("pf")
    for i in range(10):
        ch.basic_publish("", "pf", str(i).encode())
    ch.basic_qos(prefetch_count=3)
    ch.basic_consume("pf", "c")
    c.process(0.2)
    assert len(ch.deliveries) == 3
    first = [ch.deliveries.popleft() for _ in range(3)]
    ch.basic_ack(first[-1].delivery_tag, multiple=True)
    more = ch.consume_n(3)
    assert [d.body for d in more] == [b"3", b"4", b"5"]
    c.close()


def test_nack_requeue_redelivers_in_order(broker):
    c = conn(broker)
    ch = c.channel()
    ch.queue_declare("rq")
    for i in range(4):
        ch.basic_publish("", "rq", str(i).encode())
    ch.basic_consume("rq", "c")
    ds = ch.consume_n(4)
    ch.basic_nack(ds[2].delivery_tag, multiple=True, requeue=True)
    again = ch.consume_n(3)
    assert [d.body for d in again] == [b"0", b"1", b"2"]
    assert all(d.method.redelivered for d in again)
    ch.basic_reject(ds[3].delivery_tag, requeue=False)
    ch.basic_ack(0, multiple=True)
    c.process(0.1)
    assert ch.queue_declare("rq", passive=True).message_count == 0
    c.close()


def test_recover_sends_recover_ok(broker):
    c = conn(broker)
    ch = c.channel()
    ch.queue_declare("rc")
    ch.basic_publish("", "rc", b"r")
    ch.basic_consume("rc", "c")
    ch.consume_n(1)
    ch.basic_recover(requeue=True)   # RecoverOk (SURVEY A.Q11)
    d = ch.consume_n(1)[0]
    assert d.method.redelivered
    c.close()


def test_basic_get_message_count(broker):
    c = conn(broker)
    ch = c.channel()
    ch.queue_declare("g")
    for i in range(3):
        ch.basic_publish("", "g", b"m")
    time.sleep(0.05)
    d = ch.basic_get("g", no_ack=True)
    assert d.method.message_count == 2   # real remaining count (A.Q15)
    assert ch.basic_get("g", no_ack=False).method.message_count == 1
    ch.basic_get("g", no_ack=True)
    assert ch.basic_get("g") is None
    c.close()


def test_tx_commit_and_rollback(broker):
    c = conn(broker)
    ch = c.channel()
    ch.queue_declare("tx")
    ch.tx_select()
    ch.basic_publish("", "tx", b"a")
    ch.tx_rollback()
    ch.basic_publish("", "tx", b"b")
    ch.tx_commit()
    time.sleep(0.05)
    assert ch.queue_declare("tx", passive=True).message_count == 1
    c.close()


def test_channel_errors(broker):
    c = conn(broker)
    ch = c.channel()
    with pytest.raises(ChannelClosed) as e:
        ch.queue_declare("missing", passive=True)
    assert e.value.code == 404
    ch2 = c.channel()
    with pytest.raises(ChannelClosed) as e:
        ch2.queue_declare("amq.reserved")
    assert e.value.code == 403
    ch3 = c.channel()
    ch3.exchange_declare("typed", "direct")
    with pytest.raises(ChannelClosed) as e:
        ch3.exchange_declare("typed", "topic")
    assert e.value.code == 406
    ch4 = c.channel()
    with pytest.raises(ChannelClosed) as e:
        ch4.basic_ack(99)
        ch4.queue_declare("x")
    assert e.value.code == 406
    c.close()


def test_exclusive_queue_locked_and_deleted_on_close(broker):
    a = conn(broker)
    ach = a.channel()
    ach.queue_declare("excl", exclusive=True)
    b = conn(broker)
    bch = b.channel()
    with pytest.raises(ChannelClosed) as e:
        bch.basic_consume("excl", "x")
    assert e.value.code == 405
    a.close()
    time.sleep(0.1)
    bch2 = b.channel()
    with pytest.raises(ChannelClosed):
        bch2.queue_declare("excl", passive=True)
    b.close()


def test_queue_delete_if_empty_and_purge(broker):
    c = conn(broker)
    ch = c.channel()
    ch.queue_declare("dq")
    ch.basic_publish("", "dq", b"1")
    ch.basic_publish("", "dq", b"2")
    time.sleep(0.05)
    with pytest.raises(ChannelClosed):
        ch.queue_delete("dq", if_empty=True)
    ch = c.channel()
    assert ch.queue_purge("dq") == 2
    assert ch.queue_delete("dq", if_empty=True) == 0
    c.close()


def test_unknown_vhost_refused(broker):
    with pytest.raises(ConnectionClosed) as e:
        Connection(port=broker.port, vhost="/nope")
    assert e.value.code == 404
    broker.create_vhost("nope")
    c = Connection(port=broker.port, vhost="/nope")
    c.channel().queue_declare("inside")
    c.close()


def test_heartbeats_sent(broker):
    b2 = load().Broker({"port": 0, "host": "127.0.0.1", "heartbeat": 1})
    b2.start()
    try:
        c = Connection(port=b2.port, heartbeat=1)
        t0 = time.time()
        while time.time() - t0 < 2.5:
            c.process(0.3)
            c.send_heartbeat()
        assert c.heartbeats_received >= 1
        c.close()
    finally:
        b2.stop()


def test_consumer_cancel_notify_on_queue_delete(broker):
    a = conn(broker)
    ach = a.channel()
    ach.queue_declare("cn")
    ach.basic_consume("cn", "ct")
    b = conn(broker)
    b.channel().queue_delete("cn")
    a.process(0.2)
    assert "ct" in ach.cancelled
    a.close()
    b.close()


def test_channel_flow_from_client_pauses_delivery(broker):
    c = conn(broker)
    ch = c.channel()
    ch.queue_declare("fl")
    ch.basic_consume("fl", "c", no_ack=True)
    ch.flow(False)
    ch.basic_publish("", "fl", b"held")
    c.process(0.2)
    assert not ch.deliveries
    ch.flow(True)
    assert ch.consume_n(1)[0].body == b"held"
    c.close()


def test_large_message_split_into_frames(broker):
    c = conn(broker, frame_max=4096)
    ch = c.channel()
    ch.queue_declare("big")
    body = bytes(range(256)) * 1000
    ch.basic_publish("", "big", body)
    ch.basic_consume("big", "c", no_ack=True)
    assert ch.consume_n(1)[0].body == body
    c.close()


def test_access_request_replied(broker):
    from chanamq_amd.protocol.codec import Method
    c = conn(broker)
    ch = c.channel()
    r = ch._rpc("access.request", "access.request_ok", realm="/data")
    assert r.ticket == 1
    c.close()
