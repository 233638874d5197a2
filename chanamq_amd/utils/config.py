"""HOCON-subset configuration (the reference uses Typesafe Config).

Supported: ``#``/``//`` comments, ``key = value`` / ``key: value`` / ``key { ... }``,
dotted keys, quoted and unquoted strings, numbers, booleans, lists, ``${?ENV}`` and
``${path}`` substitutions, later definitions overriding earlier ones (deep merge).
Same key names and defaults as the reference; the reference's admin-port key typo
``chana.mp.amqp.admin.port`` is accepted as an alias (SURVEY A.Q26).
"""

import json
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
REFERENCE_CONF = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "conf", "reference.conf")


def _auto_wm(v, auto):
    """-1 = automatic (host broker: 1 GiB high watermark; the low one then defaults to half)."""
    return auto if v < 0 else v


def _auto_spill(v):
    """spill-bytes: -1 = automatic (1/8 of physical memory, <= 64 GiB, whole 4 MiB log blocks)."""
    if v >= 0:
        return v
    try:
        total = os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES")
    except (ValueError, OSError):
        return 0
    return (min(64 << 30, total // 8) >> 22) << 22


class ConfigError(Exception):
    pass


class _Parser:
    def __init__(self, text):
        self.s = text
        self.i = 0

    def ws(self, newlines=True):
        s = self.s
        while self.i < len(s):
            c = s[self.i]
            if c == "#" or s.startswith("//", self.i):
                while self.i < len(s) and s[self.i] != "\n":
                    self.i += 1
            elif c in " \t\r" or (newlines and c == "\n") or c == ",":
                self.i += 1
            else:
                break

    def key(self):
        self.ws()
        s = self.s
        if s[self.i] == '"':
            return self.quoted()
        m = re.compile(r"[A-Za-z0-9_\-.$]+").match(s, self.i)
        if not m:
            raise ConfigError(f"bad key at offset {self.i}: {s[self.i:self.i + 20]!r}")
        self.i = m.end()
        return m.group(0)

    def quoted(self):
        j = self.i + 1
        out = []
        while self.s[j] != '"':
            if self.s[j] == "\\":
                j += 1
                out.append({"n": "\n", "t": "\t"}.get(self.s[j], self.s[j]))
            else:
                out.append(self.s[j])
            j += 1
        self.i = j + 1
        return "".join(out)

    def value(self):
        self.ws(newlines=False)
        s = self.s
        c = s[self.i]
        if c == "{":
            self.i += 1
            obj = self.obj("}")
            return obj
        if c == "[":
            self.i += 1
            arr = []
            while True:
                self.ws()
                if s[self.i] == "]":
                    self.i += 1
                    return arr
                arr.append(self.value())
        if c == '"':
            return self.quoted()
        m = re.compile(r"[^\n,\]}#]*").match(s, self.i)
        self.i = m.end()
        raw = m.group(0)
        cut = raw.find("//")
        if cut >= 0:   # '//' starts a comment in HOCON unquoted values
            self.i -= len(raw) - cut
            raw = raw[:cut]
        return _scalar(raw.strip())

    def obj(self, close=None):
        out = {}
        while True:
            self.ws()
            if self.i >= len(self.s):
                if close:
                    raise ConfigError("unterminated object")
                return out
            if close and self.s[self.i] == close:
                self.i += 1
                return out
            k = self.key()
            self.ws(newlines=False)
            if self.s[self.i] in "=:":
                self.i += 1
            v = self.value()
            _set_path(out, k.split("."), v)


def _scalar(raw):
    if raw in ("true", "on", "yes"):
        return True
    if raw in ("false", "off", "no"):
        return False
    if raw == "null":
        return None
    if re.fullmatch(r"-?\d+", raw):
        return int(raw)
    if re.fullmatch(r"-?\d+\.\d*", raw):
        return float(raw)
    return raw


def _set_path(d, path, v):
    for p in path[:-1]:
        if not isinstance(d.get(p), dict):
            d[p] = {}
        d = d[p]
    last = path[-1]
    if isinstance(v, dict) and isinstance(d.get(last), dict):
        _merge(d[last], v)
    else:
        d[last] = v


def _merge(a, b):
    for k, v in b.items():
        if isinstance(v, dict) and isinstance(a.get(k), dict):
            _merge(a[k], v)
        else:
            a[k] = v
    return a


def parse(text):
    return _Parser(text).obj()


class Config:
    def __init__(self, tree=None):
        self.tree = tree or {}

    @classmethod
    def load(cls, files=(), overrides=None, env=True):
        tree = parse(open(REFERENCE_CONF).read())
        app = os.path.join(os.path.dirname(REFERENCE_CONF), "application.conf")
        for f in ([app] if os.path.exists(app) else []) + list(files):
            _merge(tree, parse(open(f).read()))
        cfg = cls(tree)
        cfg._resolve()
        if env:   # CHANAMQ_CHANA_MQ_AMQP_SERVER_PORT=5673 style overrides
            for k, v in os.environ.items():
                if k.startswith("CHANAMQ__"):
                    cfg.set(k[len("CHANAMQ__"):].lower().replace("__", ".").replace("_", "-"), _scalar(v))
        for k, v in (overrides or {}).items():
            cfg.set(k, v if not isinstance(v, str) else _scalar(v))
        return cfg

    def _resolve(self):
        def walk(node):
            for k, v in list(node.items()):
                if isinstance(v, dict):
                    walk(v)
                elif isinstance(v, str) and v.startswith("${") and v.endswith("}"):
                    ref = v[2:-1]
                    if ref.startswith("?"):
                        env = os.environ.get(ref[1:])
                        if env is None:
                            del node[k]
                        else:
                            node[k] = _scalar(env)
                    else:
                        node[k] = self.get(ref)
        walk(self.tree)

    def get(self, path, default=KeyError):
        d = self.tree
        for p in path.split("."):
            if not isinstance(d, dict) or p not in d:
                if path.startswith("chana.mq.amqp.admin.port"):   # reference typo alias (A.Q26)
                    alt = self.get("chana.mp.amqp.admin.port", None)
                    if alt is not None:
                        return alt
                if default is KeyError:
                    raise ConfigError(f"missing config key {path}")
                return default
            d = d[p]
        return d

    def set(self, path, value):
        _set_path(self.tree, path.split("."), value)

    def broker_config(self):
        """Keys of the native broker (csrc/core/broker.hpp BrokerConfig)."""
        g = self.get
        p12 = g("chana.mq.ssl.keystore", "")
        tls_enable = bool(g("chana.mq.amqps.server.enable")) and bool(p12 or g("chana.mq.ssl.cert", ""))
        return {
            "host": g("chana.mq.amqp.server.interface"),
            "port": int(g("chana.mq.amqp.server.port")),
            "amqp_enable": bool(g("chana.mq.amqp.server.enable")),
            "tls_port": int(g("chana.mq.amqps.server.port")),
            "tls_enable": tls_enable,
            "tls_p12": p12, "tls_p12_password": str(g("chana.mq.ssl.password", "")),
            "tls_cert": g("chana.mq.ssl.cert", ""), "tls_key": g("chana.mq.ssl.key", ""),
            "channel_max": int(g("chana.mq.amqp.connection.channel-max")),
            "frame_max": int(g("chana.mq.amqp.connection.frame-max")),
            "frame_min": int(g("chana.mq.amqp.connection.frame-min")),
            "heartbeat": int(g("chana.mq.amqp.connection.heartbeat")),
            "default_vhost": g("chana.mq.amqp.vhost.default-id"),
            "data_dir": g("chana.mq.store.dir", ""),
            "fsync": bool(g("chana.mq.store.fsync", True)),
            "mem_high_watermark": _auto_wm(int(g("chana.mq.flow.memory-high-watermark", -1)), 1 << 30),
            "mem_low_watermark": _auto_wm(int(g("chana.mq.flow.memory-low-watermark", -1)),
                                          _auto_wm(int(g("chana.mq.flow.memory-high-watermark", -1)), 1 << 30) // 2),
            "flow_channel": bool(g("chana.mq.flow.channel-flow", False)),
            "hash_wildcard": bool(g("chana.mq.routing.topic-hash-wildcard", True)),
        }

    def gpu_config(self, single=True):
        """``chana.mq.gpu.*`` -> (GpuDataPlane keyword arguments, GpuBroker keyword arguments).
        ``single``: the single-GPU server, whose step pipeline defaults to bench.py's (SDMA
        egress, whole step one graph, ingress through HSA: TCP config 2 at 5 M msgs/s p50 0.56
        vs 0.86 ms, p99 1.6 vs 6.3 ms, profiles/r6_fe2/); sharded ranks keep the engine's
        defaults unless the keys are set."""
        g = self.get
        k = "chana.mq.gpu."
        store_dir = g("chana.mq.store.dir", "")
        plane = dict(
            device=int(g(k + "device", 0)), c_max=int(g(k + "max-connections", 1024)),
            chpc=int(g(k + "channels-per-connection", 16)), q_max=int(g(k + "max-queues", 4096)),
            x_max=int(g(k + "max-exchanges", 1024)), cons_max=int(g(k + "max-consumers", 16384)),
            seg_max=int(g(k + "max-segments-per-step", 1024)), cmd_max=int(g(k + "max-commands-per-step", 131072)),
            deliv_max=int(g(k + "max-deliveries-per-step", 65536)), deliver_cap=int(g(k + "deliver-cap", 8192)),
            deliver_cap_bytes=int(g(k + "deliver-cap-bytes", 1 << 20)),
            msg_max=int(g(k + "message-table", 1 << 24)), log_bytes=int(g(k + "body-log-bytes", 64 << 30)),
            ring_pool=int(g(k + "queue-ring-pool", 1 << 28)),
            default_queue_capacity=int(g(k + "queue-capacity", 1 << 16)), ucap=int(g(k + "unacked-window", 8192)),
            ingress_cap=int(g(k + "ingress-bytes", 64 << 20)), egress_cap=int(g(k + "egress-bytes", 128 << 20)),
            carry_cap=int(g(k + "carry-bytes", 16 << 20)), tb_max=int(g(k + "topic-bindings", 4096)),
            frame_max=int(g("chana.mq.amqp.connection.frame-max")),
            hash_wildcard=bool(g("chana.mq.routing.topic-hash-wildcard", True)),
            # cold message bodies spill to this much pinned host memory once the HBM log fills
            # (-1 = auto: an eighth of the host's RAM, at most 64 GiB)
            spill_bytes=_auto_spill(int(g(k + "spill-bytes", -1))))
        # step pipeline (engine defaults unless set): the egress D2H engine (blit | sdma), the
        # overlapped ingest half, and the ingress H2D through HSA with a device-side wait
        # (h2d-hsa: single GPU, overlap off, sdma egress; bench.py's default step pipeline)
        ce = g(k + "copy-engine", "sdma" if single else None)
        if ce is not None:
            plane["copy_engine"] = {"blit": 0, "nocu": 1, "kernel": 2, "sdma": 3}[str(ce)]
        for key, name, dflt in (("overlap", "overlap", False), ("h2d-hsa", "h2d_hsa", True)):
            v = g(k + key, dflt if single else None)
            if v is not None:
                plane[name] = int(bool(v))
        if store_dir:
            plane.update(persist=1, persist_max=int(g(k + "persist-records", 1 << 16)),
                         persist_bytes=int(g(k + "persist-bytes", 256 << 20)))
        hi = int(g("chana.mq.flow.memory-high-watermark", -1))
        lo = int(g("chana.mq.flow.memory-low-watermark", -1))
        if hi < 0:   # 40% of what the broker can hold: the HBM body log + the host spill ring
            hi = int(0.4 * (plane["log_bytes"] + plane["spill_bytes"]))
        if lo < 0:
            lo = hi // 2
        broker = dict(io=str(g(k + "front-end", "pipeline")), io_threads=int(g(k + "io-threads", 4)),
                      idle_step_ms=float(g(k + "idle-step-ms", 1.0)), per_conn_read=int(g(k + "per-conn-read", 512 << 10)),
                      confirm_read=int(g(k + "confirm-read", 128 << 10)),
                      persist_group_ms=float(g(k + "persist-group-ms", 2.0)),
                      mem_high_watermark=hi, mem_low_watermark=lo)
        return plane, broker

    def __repr__(self):
        return json.dumps(self.tree, indent=1, default=str)
