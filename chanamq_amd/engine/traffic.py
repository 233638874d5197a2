"""Synthetic AMQP traffic (the PerfTest-shaped load of chana-mq-test/perf/*.js,
generated in-process: there is no network or RabbitMQ PerfTest in this image).

``publish_stream`` renders real Basic.Publish wire bytes (method + content header +
body frames) exactly as an AMQP client would put them on a socket.
"""

import struct

import numpy as np

from ..protocol.codec import Method, encode_properties, render_command


def publish_command(channel, exchange, routing_key, body, props=None, mandatory=False, frame_max=131072):
    m = Method("basic.publish", exchange=exchange, routing_key=routing_key, mandatory=mandatory)
    return render_command(channel, m, props or {}, body, frame_max)


def publish_stream(n_msgs, exchange, key_fn, body_size, channel=1, persistent=False, seed=0,
                   frame_max=131072, with_timestamp=True):
    """Concatenated publishes; ``key_fn(i) -> routing key``.  Bodies are random bytes
    (so the GPU frame scanner sees realistic false-positive candidates)."""
    rng = np.random.default_rng(seed)
    bodies = rng.integers(0, 256, size=(min(n_msgs, 64), body_size), dtype=np.uint8)
    out = []
    props = {"delivery_mode": 2 if persistent else 1}
    for i in range(n_msgs):
        if with_timestamp:
            props["timestamp"] = 1_700_000_000 + i
        out.append(publish_command(channel, exchange, key_fn(i), bodies[i % len(bodies)].tobytes(),
                                   dict(props), frame_max=frame_max))
    return b"".join(out)


def split_stream(data: bytes, parts: int, seed=0):
    """Split a byte stream at arbitrary (non frame-aligned) offsets: TCP reads."""
    n = len(data)
    if parts <= 1:
        return [data]
    rng = np.random.default_rng(seed)
    cuts = sorted(set(int(x) for x in rng.integers(1, n, size=parts - 1)))
    bounds = [0] + cuts + [n]
    return [data[bounds[i]:bounds[i + 1]] for i in range(len(bounds) - 1)]


def even_split(data: bytes, parts: int):
    """``parts`` chunks of near-equal size (frame boundaries ignored)."""
    n = len(data)
    step = -(-n // parts)
    return [data[i * step:(i + 1) * step] for i in range(parts)]


def ack_frame(channel, tag, multiple=True):
    return render_command(channel, Method("basic.ack", delivery_tag=tag, multiple=multiple))


def heartbeat():
    return struct.pack(">BHI", 8, 0, 0) + b"\xce"


__all__ = ["publish_command", "publish_stream", "split_stream", "even_split", "ack_frame", "heartbeat",
           "encode_properties"]
