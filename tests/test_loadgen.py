"""Native PerfTest-style load generator smoke test (host path, short)."""
from chanamq_amd.broker import load


def test_loadgen_roundtrip():
    core = load()
    b = core.Broker({"port": 0, "host": "127.0.0.1", "heartbeat": 0})
    b.start()
    try:
        r = core.run_load(dict(port=b.port, producers=1, consumers=1, msg_size=64, seconds=0.5, rate=20000))
        assert r["error"] == "" and r["received"] > 1000 and r["p50_us"] > 0
        r = core.run_load(dict(port=b.port, producers=2, consumers=2, msg_size=0, seconds=0.5, auto_ack=False,
                               prefetch=100, queue="m.q", exchange="m.x", queues=2))
        assert r["error"] == "" and r["received"] > 100
        # redelivery storm: every 2nd settle of each consumer is Nack(multiple, requeue)
        r = core.run_load(dict(port=b.port, producers=2, consumers=2, msg_size=32, seconds=0.7, auto_ack=False,
                               prefetch=50, queue="s.q", exchange="s.x", nack_every=2))
        assert r["error"] == "" and r["requeued"] > 0 and r["redelivered"] > 0
        assert r["redelivered"] <= r["received"]
    finally:
        b.stop()
