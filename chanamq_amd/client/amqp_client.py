"""Minimal blocking AMQP 0-9-1 client built on the golden codec.

Used by the conversation tests (the reference's SimplePublisher / SimpleConsumer
scenarios, chana-mq-test/src/main/scala/chana/mq/test/*.scala) and by the host-path
load generator.  ``pika`` is not installed in this image, so this is our own client.
"""

import collections
import select
import socket
import ssl as _ssl
import struct
import time

from ..protocol import constants as C
from ..protocol.codec import (CommandAssembler, FrameParser, Method, encode_frame, encode_method_frame,
                              render_command)


class ChannelClosed(Exception):
    def __init__(self, code, text, cls=0, mid=0):
        super().__init__(f"{code} {text}")
        self.code, self.text = code, text


class ConnectionClosed(ChannelClosed):
    pass


class Delivery:
    __slots__ = ("method", "props", "body", "channel")

    def __init__(self, channel, method, props, body):
        self.channel, self.method, self.props, self.body = channel, method, props, body

    @property
    def delivery_tag(self):
        return self.method.delivery_tag

    def __repr__(self):
        return f"Delivery({self.method.name}, tag={getattr(self.method, 'delivery_tag', None)}, {len(self.body)}B)"


class Channel:
    def __init__(self, conn, number):
        self.conn = conn
        self.number = number
        self.inbox = collections.deque()      # replies for synchronous methods
        self.deliveries = collections.deque()  # Basic.Deliver / GetOk
        self.returns = collections.deque()
        self.confirms = collections.deque()   # (tag, multiple, is_ack)
        self.closed = None
        self.flow_active = True
        self.cancelled = []
        self.published = 0
        self.confirmed_upto = 0   # highest confirmed publish sequence seen (across waits)
        self.confirm_mode = False
        self.consumer_tags = set()   # tags whose Basic.ConsumeOk arrived (strict ordering check)

    # ---------------------------------------------------------------- plumbing
    def _send(self, name, **args):
        self.conn._send_method(self.number, Method(name, **args))

    def _rpc(self, name, reply, **args):
        self._send(name, **args)
        return self.conn._wait(lambda: self._pop_reply(reply), self)

    def _pop_reply(self, reply):
        if self.closed:
            raise self.closed
        for i, m in enumerate(self.inbox):
            if m.name == reply:
                del self.inbox[i]
                return m
        return None

    # ---------------------------------------------------------------- api
    def exchange_declare(self, exchange, type="direct", passive=False, durable=False, auto_delete=False,
                         internal=False, arguments=None, nowait=False):
        args = dict(exchange=exchange, type=type, passive=passive, durable=durable, auto_delete=auto_delete,
                    internal=internal, nowait=nowait, arguments=arguments or {})
        if nowait:
            return self._send("exchange.declare", **args)
        return self._rpc("exchange.declare", "exchange.declare_ok", **args)

    def exchange_delete(self, exchange, if_unused=False):
        return self._rpc("exchange.delete", "exchange.delete_ok", exchange=exchange, if_unused=if_unused)

    def exchange_bind(self, destination, source, routing_key=""):
        return self._rpc("exchange.bind", "exchange.bind_ok", destination=destination, source=source,
                         routing_key=routing_key)

    def exchange_unbind(self, destination, source, routing_key=""):
        return self._rpc("exchange.unbind", "exchange.unbind_ok", destination=destination, source=source,
                         routing_key=routing_key)

    def queue_declare(self, queue="", passive=False, durable=False, exclusive=False, auto_delete=False,
                      arguments=None):
        return self._rpc("queue.declare", "queue.declare_ok", queue=queue, passive=passive, durable=durable,
                         exclusive=exclusive, auto_delete=auto_delete, arguments=arguments or {})

    def queue_bind(self, queue, exchange, routing_key="", arguments=None):
        return self._rpc("queue.bind", "queue.bind_ok", queue=queue, exchange=exchange, routing_key=routing_key,
                         arguments=arguments or {})

    def queue_unbind(self, queue, exchange, routing_key=""):
        return self._rpc("queue.unbind", "queue.unbind_ok", queue=queue, exchange=exchange, routing_key=routing_key)

    def queue_purge(self, queue):
        return self._rpc("queue.purge", "queue.purge_ok", queue=queue).message_count

    def queue_delete(self, queue, if_unused=False, if_empty=False):
        return self._rpc("queue.delete", "queue.delete_ok", queue=queue, if_unused=if_unused,
                         if_empty=if_empty).message_count

    def basic_qos(self, prefetch_count=0, prefetch_size=0, global_=False):
        return self._rpc("basic.qos", "basic.qos_ok", prefetch_size=prefetch_size, prefetch_count=prefetch_count,
                         global_=global_)

    def basic_consume(self, queue, consumer_tag="", no_ack=False, exclusive=False):
        return self._rpc("basic.consume", "basic.consume_ok", queue=queue, consumer_tag=consumer_tag,
                         no_ack=no_ack, exclusive=exclusive).consumer_tag

    def basic_cancel(self, consumer_tag):
        return self._rpc("basic.cancel", "basic.cancel_ok", consumer_tag=consumer_tag)

    def basic_publish(self, exchange, routing_key, body, properties=None, mandatory=False, immediate=False):
        m = Method("basic.publish", exchange=exchange, routing_key=routing_key, mandatory=mandatory,
                   immediate=immediate)
        self.conn._send_raw(render_command(self.number, m, properties or {}, body, self.conn.frame_max))
        if self.confirm_mode:   # publish sequence numbers start at 1 with Confirm.Select
            self.published += 1

    def basic_get(self, queue, no_ack=False):
        self._send("basic.get", queue=queue, no_ack=no_ack)

        def pred():
            if self.closed:
                raise self.closed
            for i, m in enumerate(self.inbox):
                if m.name == "basic.get_empty":
                    del self.inbox[i]
                    return (None,)
            for i, d in enumerate(self.deliveries):
                if d.method.name == "basic.get_ok":
                    del self.deliveries[i]
                    return (d,)
            return None
        return self.conn._wait(pred, self)[0]

    def basic_get_many(self, queue, n, no_ack=True):
        """``n`` pipelined Basic.Gets in one write (the server answers them in order): the
        GetOk deliveries, and how many came back GetEmpty."""
        self.conn._send_raw(encode_method_frame(self.number, Method("basic.get", queue=queue, no_ack=no_ack)) * n)
        state = {"ok": [], "empty": 0}

        def pred():
            if self.closed:
                raise self.closed
            for i in range(len(self.inbox) - 1, -1, -1):
                if self.inbox[i].name == "basic.get_empty":
                    del self.inbox[i]
                    state["empty"] += 1
            keep = collections.deque()
            while self.deliveries:
                d = self.deliveries.popleft()
                (state["ok"] if d.method.name == "basic.get_ok" else keep).append(d)
            self.deliveries.extend(keep)
            return True if len(state["ok"]) + state["empty"] >= n else None
        self.conn._wait(pred, self)
        return state["ok"], state["empty"]

    def basic_ack(self, delivery_tag, multiple=False):
        self._send("basic.ack", delivery_tag=delivery_tag, multiple=multiple)

    def basic_nack(self, delivery_tag, multiple=False, requeue=True):
        self._send("basic.nack", delivery_tag=delivery_tag, multiple=multiple, requeue=requeue)

    def basic_reject(self, delivery_tag, requeue=True):
        self._send("basic.reject", delivery_tag=delivery_tag, requeue=requeue)

    def basic_recover(self, requeue=True):
        return self._rpc("basic.recover", "basic.recover_ok", requeue=requeue)

    def confirm_select(self):
        self.confirm_mode = True
        return self._rpc("confirm.select", "confirm.select_ok")

    def tx_select(self):
        return self._rpc("tx.select", "tx.select_ok")

    def tx_commit(self):
        return self._rpc("tx.commit", "tx.commit_ok")

    def tx_rollback(self):
        return self._rpc("tx.rollback", "tx.rollback_ok")

    def flow(self, active):
        return self._rpc("channel.flow", "channel.flow_ok", active=active)

    def wait_for_confirms(self, timeout=10.0):
        """Block until every publish so far is acked; returns False if any was nacked."""
        state = {"nacked": False}

        def pred():
            while self.confirms:
                tag, multiple, ok = self.confirms.popleft()
                if not ok:
                    state["nacked"] = True
                self.confirmed_upto = max(self.confirmed_upto, tag)
            return True if self.confirmed_upto >= self.published else None
        self.conn._wait(pred, self, timeout)
        return not state["nacked"]

    def consume_n(self, n, timeout=10.0):
        out = []

        def pred():
            while self.deliveries and len(out) < n:
                out.append(self.deliveries.popleft())
            return True if len(out) >= n else None
        self.conn._wait(pred, self, timeout)
        return out

    def close(self):
        if self.closed:
            return
        self._rpc("channel.close", "channel.close_ok", reply_code=200, reply_text="bye")
        self.closed = ChannelClosed(200, "closed")
        self.conn.channels.pop(self.number, None)


class Connection:
    def __init__(self, host="127.0.0.1", port=5672, vhost="/", user="guest", password="guest", heartbeat=0,
                 frame_max=131072, tls=False, timeout=10.0, capabilities=None, strict=False):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        if tls:
            ctx = _ssl.create_default_context()
            ctx.check_hostname = False
            ctx.verify_mode = _ssl.CERT_NONE
            self.sock = ctx.wrap_socket(self.sock)
        self.timeout = timeout
        self.parser = FrameParser()
        self.assemblers = collections.defaultdict(CommandAssembler)
        self.channels = {}
        self.conn_inbox = collections.deque()
        self.closed = None
        self.blocked = False
        self.server_properties = None
        self.frame_max = frame_max
        self.heartbeats_received = 0
        # strict: record what a strict client (the Java client's "Unsolicited delivery")
        # rejects -- a Basic.Deliver for a consumer tag whose ConsumeOk has not arrived yet
        self.strict = strict
        self.violations = []
        self._next_ch = 1
        self._wbuf = bytearray()
        self._send_raw(C.PROTOCOL_HEADER)
        start = self._wait_conn("connection.start")
        self.server_properties = start.server_properties
        caps = capabilities or {"publisher_confirms": True, "connection.blocked": True,
                                "consumer_cancel_notify": True, "basic.nack": True}
        self._send_method(0, Method("connection.start_ok", client_properties={"product": "chanamq-test",
                                                                              "capabilities": caps},
                                    mechanism="PLAIN", response=b"\x00" + user.encode() + b"\x00" + password.encode(),
                                    locale="en_US"))
        tune = self._wait_conn("connection.tune")
        fm = min(frame_max, tune.frame_max) if tune.frame_max else frame_max
        self.frame_max = fm
        self.heartbeat = heartbeat
        self._send_method(0, Method("connection.tune_ok", channel_max=tune.channel_max or 2047, frame_max=fm,
                                    heartbeat=heartbeat))
        self._send_method(0, Method("connection.open", virtual_host=vhost))
        self._wait_conn("connection.open_ok")

    # ---------------------------------------------------------------- io
    def _send_raw(self, data):
        self.sock.sendall(data)

    def _send_method(self, ch, m):
        self._send_raw(encode_method_frame(ch, m))

    def _pump(self, timeout):
        """Read what is available within ``timeout`` seconds and dispatch it.

        The socket itself always stays in blocking mode with ``self.timeout``
        (so ``sendall`` never sees ``EAGAIN``); the read window is enforced
        with ``select``.  A window of <= 0 is a poll.  TLS sockets can hold
        decrypted bytes that ``select`` does not see, so ``pending()`` is
        checked first.
        """
        pending = isinstance(self.sock, _ssl.SSLSocket) and self.sock.pending() > 0
        if not pending:
            try:
                ready, _, _ = select.select([self.sock], [], [], max(0.0, timeout))
            except (OSError, ValueError):
                ready = [self.sock]   # closed fd: let recv report it
            if not ready:
                return
        try:
            data = self.sock.recv(1 << 20)
        except (socket.timeout, BlockingIOError, InterruptedError, _ssl.SSLWantReadError):
            return
        if not data:
            if self.closed is None:
                self.closed = ConnectionClosed(320, "socket closed by peer")
            raise self.closed
        for fr in self.parser.feed(data):
            if fr.type == C.FRAME_HEARTBEAT:
                self.heartbeats_received += 1
                continue
            cmd = self.assemblers[fr.channel].feed(fr)
            if cmd is not None:
                self._on_command(cmd)

    def _on_command(self, cmd):
        m = cmd.method
        if cmd.channel == 0:
            if m.name == "connection.close":
                self.closed = ConnectionClosed(m.reply_code, m.reply_text)
                try:
                    self._send_method(0, Method("connection.close_ok"))
                except OSError:
                    pass
            elif m.name == "connection.blocked":
                self.blocked = True
            elif m.name == "connection.unblocked":
                self.blocked = False
            else:
                self.conn_inbox.append(m)
            return
        ch = self.channels.get(cmd.channel)
        if ch is None:
            return
        if m.name == "basic.consume_ok":
            ch.consumer_tags.add(m.consumer_tag)
        elif m.name == "basic.deliver" and self.strict and m.consumer_tag not in ch.consumer_tags:
            self.violations.append(f"unsolicited delivery: tag {m.consumer_tag!r} before its consume_ok")
        if m.name in ("basic.deliver", "basic.get_ok"):
            ch.deliveries.append(Delivery(cmd.channel, m, cmd.props, cmd.body))
        elif m.name == "basic.return":
            ch.returns.append(Delivery(cmd.channel, m, cmd.props, cmd.body))
        elif m.name in ("basic.ack", "basic.nack") and ch.confirm_mode:
            ch.confirms.append((m.delivery_tag, m.multiple, m.name == "basic.ack"))
        elif m.name == "channel.close":
            ch.closed = ChannelClosed(m.reply_code, m.reply_text)
            self._send_method(cmd.channel, Method("channel.close_ok"))
            self.channels.pop(cmd.channel, None)
        elif m.name == "channel.flow":
            ch.flow_active = m.active
            self._send_method(cmd.channel, Method("channel.flow_ok", active=m.active))
        elif m.name == "basic.cancel":
            ch.cancelled.append(m.consumer_tag)
        else:
            ch.inbox.append(m)

    def _wait(self, pred, ch=None, timeout=None):
        deadline = time.time() + (timeout or self.timeout)
        while True:
            r = pred()
            if r is not None:
                return r
            if self.closed:
                raise self.closed
            if ch is not None and ch.closed:
                raise ch.closed
            left = deadline - time.time()
            if left <= 0:
                raise TimeoutError("timed out waiting for broker")
            self._pump(min(left, 0.5))

    def _wait_conn(self, name):
        def pred():
            for i, m in enumerate(self.conn_inbox):
                if m.name == name:
                    del self.conn_inbox[i]
                    return m
            return None
        return self._wait(pred)

    def process(self, seconds=0.05):
        """Pump incoming frames for a while (heartbeats, deliveries)."""
        end = time.time() + seconds
        while time.time() < end:
            self._pump(max(0.0, end - time.time()))

    def send_heartbeat(self):
        self._send_raw(encode_frame(C.FRAME_HEARTBEAT, 0, b""))

    # ---------------------------------------------------------------- api
    def channel(self, number=None):
        n = number or self._next_ch
        self._next_ch = max(self._next_ch, n) + 1
        ch = Channel(self, n)
        self.channels[n] = ch
        ch._rpc("channel.open", "channel.open_ok")
        return ch

    def close(self):
        if self.closed:
            try:
                self.sock.close()
            finally:
                return
        try:
            self._send_method(0, Method("connection.close", reply_code=200, reply_text="bye"))
            self._wait_conn("connection.close_ok")
        except (OSError, ChannelClosed, TimeoutError):
            pass
        self.closed = ConnectionClosed(200, "closed")
        self.sock.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
