"""Config system (same keys/defaults as the reference) and the admin REST API."""

import json
import os
import subprocess
import sys
import time
import urllib.request

import pytest

from chanamq_amd.broker import load
from chanamq_amd.client import Connection, ConnectionClosed
from chanamq_amd.server.admin import AdminServer
from chanamq_amd.utils.config import Config, parse


def test_reference_defaults():
    c = Config.load(env=False)
    assert c.get("chana.mq.amqp.connection.frame-max") == 131072
    assert c.get("chana.mq.amqp.connection.frame-min") == 4096
    assert c.get("chana.mq.amqp.connection.heartbeat") == 30
    assert c.get("chana.mq.amqp.connection.channel-max") == 0
    assert c.get("chana.mq.amqp.server.port") == 5672
    assert c.get("chana.mq.amqps.server.port") == 5671
    assert c.get("chana.mq.amqp.vhost.default-id") == "AMQ.DEFAULT"
    assert c.get("chana.mq.amqp.vhost.seperator") == "-_."
    assert c.get("chana.mq.internal.timeout") == 20
    assert c.get("chana.mq.message.inactive") == 3600
    assert c.get("chana.mq.cassandra.pass-through.hosts") == ["localhost"]
    assert c.get("chana.mq.amqp.admin.port") == 15672


def test_hocon_subset_and_admin_typo_alias(tmp_path):
    f = tmp_path / "prod.conf"
    f.write_text('chana.mp.amqp.admin {\n port = 16000 // typo key of the deploy confs\n}\n'
                 'chana.mq.amqp.connection { heartbeat: 10, frame-max = 65536 }\n# comment\n'
                 'a.b = "x y"\nlist = [1, 2, "three"]\n')
    c = Config.load([str(f)], overrides={"chana.mq.amqp.server.port": "5800"}, env=False)
    c.tree.get("chana", {}).get("mq", {}).get("amqp", {}).pop("admin", None)
    assert c.get("chana.mq.amqp.admin.port") == 16000
    assert c.get("chana.mq.amqp.connection.heartbeat") == 10
    assert c.get("chana.mq.amqp.connection.frame-min") == 4096
    assert c.get("a.b") == "x y" and c.get("list") == [1, 2, "three"]
    assert c.get("chana.mq.amqp.server.port") == 5800
    assert parse("x { y { z = 1 } }\nx.y.w = 2") == {"x": {"y": {"z": 1, "w": 2}}}


def test_admin_vhost_put_delete_and_stats():
    core = load()
    b = core.Broker({"port": 0, "host": "127.0.0.1", "heartbeat": 0})
    b.start()
    admin = AdminServer(b, 0).start()
    try:
        base = f"http://127.0.0.1:{admin.port}"
        r = urllib.request.urlopen(base + "/admin/vhost/put/tenant1/")
        assert r.status == 200 and r.headers["Access-Control-Allow-Origin"] == "*"
        c = Connection(port=b.port, vhost="tenant1")
        c.channel().queue_declare("q")
        c.close()
        assert urllib.request.urlopen(base + "/admin/vhost/delete/tenant1").status == 200
        with pytest.raises(ConnectionClosed):
            Connection(port=b.port, vhost="tenant1")
        s = json.loads(urllib.request.urlopen(base + "/admin/stats").read())
        assert "published" in s and "connections" in s
        qs = json.loads(urllib.request.urlopen(base + "/admin/queues").read())
        assert any(q["name"] == "q" for q in qs)
    finally:
        admin.stop()
        b.stop()


def test_server_launcher_subprocess(tmp_path):
    env = dict(os.environ)
    env["PYTHONPATH"] = os.getcwd()
    p = subprocess.Popen([sys.executable, "-m", "chanamq_amd.server", "--set", "chana.mq.amqp.server.port=5779",
                          "--set", "chana.mq.amqp.admin.port=15779", "--set", "chana.mq.amqp.server.interface=127.0.0.1",
                          "--set", f"chana.mq.store.dir={tmp_path}", "--stats-interval", "0.5"],
                         env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    try:
        for _ in range(100):
            try:
                c = Connection(port=5779)
                break
            except OSError:
                time.sleep(0.1)
        ch = c.channel()
        ch.queue_declare("launch")
        ch.basic_publish("", "launch", b"hi")
        time.sleep(1.2)
        c.close()
    finally:
        p.terminate()
        out = p.communicate(timeout=20)[0].decode()
    assert "published msgs" in out and "delivered msgs" in out


def test_sharded_rank_reads_gpu_config(tmp_path):
    """server/sharded.py sizes every rank from chana.mq.gpu.* (it used to
    hard-code a 2 GB body log), command-line flags win, spill is on by default."""
    import argparse

    from chanamq_amd.server.sharded import sharded_plane_config
    from chanamq_amd.utils.config import Config
    f = tmp_path / "rank.conf"
    f.write_text("chana.mq.gpu { body-log-bytes = 68719476736, message-table = 134217728, max-connections = 512 }\n")
    cfg = Config.load([str(f)], {"chana.mq.gpu.io-threads": "6"})
    args = argparse.Namespace(c_max=None, idle_step_ms=None, io_threads=None)
    plane, broker = sharded_plane_config(cfg, args, world=8, rank=3, pipeline=True)
    assert plane["log_bytes"] == 64 << 30 and plane["msg_max"] == 1 << 27 and plane["c_max"] == 512
    assert plane["world"] == 8 and plane["rank"] == 3 and plane["native_xchg"] == 1 and plane["links"] == 1
    assert "device" not in plane and plane["seg_max"] <= plane["c_max"]
    assert plane["spill_bytes"] > 0 and plane["spill_bytes"] % (4 << 20) == 0
    assert broker["io_threads"] == 6 and "io" not in broker
    assert broker["mem_high_watermark"] == int(0.4 * (plane["log_bytes"] + plane["spill_bytes"]))
    args = argparse.Namespace(c_max=64, idle_step_ms=0.5, io_threads=2)
    plane, broker = sharded_plane_config(cfg, args, world=2, rank=0, pipeline=False)
    assert plane["c_max"] == 64 and plane["native_xchg"] == 0 and broker["idle_step_ms"] == 0.5


def test_gpu_step_pipeline_keys(tmp_path):
    """chana.mq.gpu.copy-engine / overlap / h2d-hsa: the single-GPU server defaults to
    bench.py's step pipeline, sharded ranks to the engine's; set keys win."""
    from chanamq_amd.utils.config import Config
    plane, _ = Config.load([], {}).gpu_config()   # the single-GPU server: bench.py's pipeline
    assert plane["copy_engine"] == 3 and plane["overlap"] == 0 and plane["h2d_hsa"] == 1
    plane, _ = Config.load([], {}).gpu_config(single=False)   # sharded ranks: the engine's
    assert not {"copy_engine", "overlap", "h2d_hsa"} & set(plane)
    f = tmp_path / "p.conf"
    f.write_text("chana.mq.gpu { copy-engine = blit, overlap = true, h2d-hsa = false }\n")
    plane, _ = Config.load([str(f)], {}).gpu_config()
    assert plane["copy_engine"] == 0 and plane["overlap"] == 1 and plane["h2d_hsa"] == 0
