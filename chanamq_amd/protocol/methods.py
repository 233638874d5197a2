"""AMQP 0-9-1 method table (every class/method the reference decodes).

One declarative table drives both the Python golden codec (``codec.py``) and the
C++ method table (``csrc/core/methods.hpp`` is kept in the same order; a test
cross-checks them).  Reference counterparts: chana-mq-base/.../method/*.scala
(Connection.scala:46-226, Channel.scala:39-121, Access.scala:18-53,
Exchange.scala:23-154, Queue.scala:44-203, Basic.scala:31-318,
Confirm.scala:10-44, Tx.scala:34-106).

Field types: bit, octet, short, long, longlong, shortstr, longstr, table, timestamp.
"""

from collections import namedtuple

MethodSpec = namedtuple("MethodSpec", "class_id method_id name fields content synchronous")

_T = []


def _m(cid, mid, name, fields=(), content=False, sync=False):
    _T.append(MethodSpec(cid, mid, name, tuple(fields), content, sync))


# ---- connection (10)
_m(10, 10, "connection.start", [("version_major", "octet"), ("version_minor", "octet"),
                                 ("server_properties", "table"), ("mechanisms", "longstr"),
                                 ("locales", "longstr")], sync=True)
_m(10, 11, "connection.start_ok", [("client_properties", "table"), ("mechanism", "shortstr"),
                                   ("response", "longstr"), ("locale", "shortstr")])
_m(10, 20, "connection.secure", [("challenge", "longstr")], sync=True)
_m(10, 21, "connection.secure_ok", [("response", "longstr")])
_m(10, 30, "connection.tune", [("channel_max", "short"), ("frame_max", "long"), ("heartbeat", "short")], sync=True)
_m(10, 31, "connection.tune_ok", [("channel_max", "short"), ("frame_max", "long"), ("heartbeat", "short")])
_m(10, 40, "connection.open", [("virtual_host", "shortstr"), ("capabilities", "shortstr"), ("insist", "bit")], sync=True)
_m(10, 41, "connection.open_ok", [("known_hosts", "shortstr")])
_m(10, 50, "connection.close", [("reply_code", "short"), ("reply_text", "shortstr"),
                                ("class_id", "short"), ("method_id", "short")], sync=True)
_m(10, 51, "connection.close_ok")
_m(10, 60, "connection.blocked", [("reason", "shortstr")])
_m(10, 61, "connection.unblocked")
# ---- channel (20)
_m(20, 10, "channel.open", [("out_of_band", "shortstr")], sync=True)
_m(20, 11, "channel.open_ok", [("channel_id", "longstr")])
_m(20, 20, "channel.flow", [("active", "bit")], sync=True)
_m(20, 21, "channel.flow_ok", [("active", "bit")])
_m(20, 40, "channel.close", [("reply_code", "short"), ("reply_text", "shortstr"),
                             ("class_id", "short"), ("method_id", "short")], sync=True)
_m(20, 41, "channel.close_ok")
# ---- access (30)
_m(30, 10, "access.request", [("realm", "shortstr"), ("exclusive", "bit"), ("passive", "bit"),
                              ("active", "bit"), ("write", "bit"), ("read", "bit")], sync=True)
_m(30, 11, "access.request_ok", [("ticket", "short")])
# ---- exchange (40)
_m(40, 10, "exchange.declare", [("ticket", "short"), ("exchange", "shortstr"), ("type", "shortstr"),
                                ("passive", "bit"), ("durable", "bit"), ("auto_delete", "bit"),
                                ("internal", "bit"), ("nowait", "bit"), ("arguments", "table")], sync=True)
_m(40, 11, "exchange.declare_ok")
_m(40, 20, "exchange.delete", [("ticket", "short"), ("exchange", "shortstr"), ("if_unused", "bit"),
                               ("nowait", "bit")], sync=True)
_m(40, 21, "exchange.delete_ok")
_m(40, 30, "exchange.bind", [("ticket", "short"), ("destination", "shortstr"), ("source", "shortstr"),
                             ("routing_key", "shortstr"), ("nowait", "bit"), ("arguments", "table")], sync=True)
_m(40, 31, "exchange.bind_ok")
_m(40, 40, "exchange.unbind", [("ticket", "short"), ("destination", "shortstr"), ("source", "shortstr"),
                               ("routing_key", "shortstr"), ("nowait", "bit"), ("arguments", "table")], sync=True)
_m(40, 51, "exchange.unbind_ok")
# ---- queue (50)
_m(50, 10, "queue.declare", [("ticket", "short"), ("queue", "shortstr"), ("passive", "bit"),
                             ("durable", "bit"), ("exclusive", "bit"), ("auto_delete", "bit"),
                             ("nowait", "bit"), ("arguments", "table")], sync=True)
_m(50, 11, "queue.declare_ok", [("queue", "shortstr"), ("message_count", "long"), ("consumer_count", "long")])
_m(50, 20, "queue.bind", [("ticket", "short"), ("queue", "shortstr"), ("exchange", "shortstr"),
                          ("routing_key", "shortstr"), ("nowait", "bit"), ("arguments", "table")], sync=True)
_m(50, 21, "queue.bind_ok")
_m(50, 30, "queue.purge", [("ticket", "short"), ("queue", "shortstr"), ("nowait", "bit")], sync=True)
_m(50, 31, "queue.purge_ok", [("message_count", "long")])
_m(50, 40, "queue.delete", [("ticket", "short"), ("queue", "shortstr"), ("if_unused", "bit"),
                            ("if_empty", "bit"), ("nowait", "bit")], sync=True)
_m(50, 41, "queue.delete_ok", [("message_count", "long")])
_m(50, 50, "queue.unbind", [("ticket", "short"), ("queue", "shortstr"), ("exchange", "shortstr"),
                            ("routing_key", "shortstr"), ("arguments", "table")], sync=True)
_m(50, 51, "queue.unbind_ok")
# ---- basic (60)
_m(60, 10, "basic.qos", [("prefetch_size", "long"), ("prefetch_count", "short"), ("global_", "bit")], sync=True)
_m(60, 11, "basic.qos_ok")
_m(60, 20, "basic.consume", [("ticket", "short"), ("queue", "shortstr"), ("consumer_tag", "shortstr"),
                             ("no_local", "bit"), ("no_ack", "bit"), ("exclusive", "bit"),
                             ("nowait", "bit"), ("arguments", "table")], sync=True)
_m(60, 21, "basic.consume_ok", [("consumer_tag", "shortstr")])
_m(60, 30, "basic.cancel", [("consumer_tag", "shortstr"), ("nowait", "bit")], sync=True)
_m(60, 31, "basic.cancel_ok", [("consumer_tag", "shortstr")])
_m(60, 40, "basic.publish", [("ticket", "short"), ("exchange", "shortstr"), ("routing_key", "shortstr"),
                             ("mandatory", "bit"), ("immediate", "bit")], content=True)
_m(60, 50, "basic.return", [("reply_code", "short"), ("reply_text", "shortstr"), ("exchange", "shortstr"),
                            ("routing_key", "shortstr")], content=True)
_m(60, 60, "basic.deliver", [("consumer_tag", "shortstr"), ("delivery_tag", "longlong"),
                             ("redelivered", "bit"), ("exchange", "shortstr"), ("routing_key", "shortstr")],
   content=True)
_m(60, 70, "basic.get", [("ticket", "short"), ("queue", "shortstr"), ("no_ack", "bit")], sync=True)
_m(60, 71, "basic.get_ok", [("delivery_tag", "longlong"), ("redelivered", "bit"), ("exchange", "shortstr"),
                            ("routing_key", "shortstr"), ("message_count", "long")], content=True)
_m(60, 72, "basic.get_empty", [("cluster_id", "shortstr")])
_m(60, 80, "basic.ack", [("delivery_tag", "longlong"), ("multiple", "bit")])
_m(60, 90, "basic.reject", [("delivery_tag", "longlong"), ("requeue", "bit")])
_m(60, 100, "basic.recover_async", [("requeue", "bit")])
_m(60, 110, "basic.recover", [("requeue", "bit")], sync=True)
_m(60, 111, "basic.recover_ok")
_m(60, 120, "basic.nack", [("delivery_tag", "longlong"), ("multiple", "bit"), ("requeue", "bit")])
# ---- confirm (85)
_m(85, 10, "confirm.select", [("nowait", "bit")], sync=True)
_m(85, 11, "confirm.select_ok")
# ---- tx (90)
_m(90, 10, "tx.select", sync=True)
_m(90, 11, "tx.select_ok")
_m(90, 20, "tx.commit", sync=True)
_m(90, 21, "tx.commit_ok")
_m(90, 30, "tx.rollback", sync=True)
_m(90, 31, "tx.rollback_ok")

METHODS = tuple(_T)
BY_ID = {(m.class_id, m.method_id): m for m in METHODS}
BY_NAME = {m.name: m for m in METHODS}

# Basic content-header properties, in wire order (BasicProperties.scala:42-96).
BASIC_PROPERTIES = (
    ("content_type", "shortstr"),
    ("content_encoding", "shortstr"),
    ("headers", "table"),
    ("delivery_mode", "octet"),
    ("priority", "octet"),
    ("correlation_id", "shortstr"),
    ("reply_to", "shortstr"),
    ("expiration", "shortstr"),
    ("message_id", "shortstr"),
    ("timestamp", "timestamp"),
    ("type", "shortstr"),
    ("user_id", "shortstr"),
    ("app_id", "shortstr"),
    ("cluster_id", "shortstr"),
)
