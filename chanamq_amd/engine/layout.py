"""Host mirrors of the data-plane structs (csrc/kernels/dp_common.h) and hashes.

Every numpy dtype here must match ``sizeof`` reported by ``Engine.info()['sizeof']``;
tests/test_layout.py and the GPU tests check that.
"""

import numpy as np

SEG_IN = np.dtype([("conn", "<u4"), ("len", "<u4"), ("src", "<u8")])
SEG_OUT = np.dtype([("conn", "<u4"), ("status", "<u4"), ("consumed", "<u4"), ("carry", "<u4"),
                    ("ncmds", "<u4"), ("err_off", "<u4"), ("pad", "<u4", 2)])
CTRL_REC = np.dtype([("conn", "<u4"), ("off", "<u4"), ("len", "<u4"), ("seg", "<u4")])
CONN_OUT = np.dtype([("off", "<u4"), ("len", "<u4")])
# cross-rank publish record (dp_common.h RDesc); payload = [exchange][routing key][props][body]
RDESC = np.dtype([("pay_off", "<u4"), ("body_len", "<u4"), ("props_len", "<u4"), ("exch", "<i4"),
                  ("flags", "<u4"), ("ex_len", "u1"), ("rk_len", "u1"), ("pad0", "<u2"),
                  ("expire_ms", "<i8"), ("ts_ms", "<i8"), ("xid", "<u8"), ("tq", "<u4"), ("pad", "<u4", 3)])
MF_PERSIST, MF_MANDATORY, MF_IMMEDIATE, MF_HAS_TS, MF_IMPORTED = 1, 2, 4, 8, 16
MF_RESTORE, MF_REDELIVERED, MF_ONEQ, MF_SLOTFMT, MF_HOSTPUB = 32, 64, 128, 256, 512
# persistence records (dp_common.h PersistHdr / ConsumedRec)
PERSIST_HDR = np.dtype([("msg_id", "<i8"), ("ts_ms", "<i8"), ("qpos", "<u8"), ("expire_ms", "<i8"), ("q", "<u4"),
                        ("body_len", "<u4"), ("props_len", "<u2"), ("ex_len", "u1"), ("rk_len", "u1"),
                        ("size", "<u4")])
CONSUMED_REC = np.dtype([("msg_id", "<i8"), ("qpos", "<u8"), ("q", "<u4"), ("kind", "<u4"), ("pad", "<u4", 2)])
# a queue ring grown by the device (step_abi.h RingMove)
RING_MOVE = np.dtype([("q", "<u4"), ("pad", "<u4"), ("old_off", "<u8"), ("old_mask", "<u8"), ("new_off", "<u8"),
                      ("new_mask", "<u8"), ("head", "<u8"), ("tail", "<u8")])
assert PERSIST_HDR.itemsize == 48 and CONSUMED_REC.itemsize == 32

# per-channel unacked window slot (dp_common.h USlot)
USLOT = np.dtype([("state", "<u4"), ("msg", "<u4"), ("q", "<u4"), ("cons", "<u4"), ("qpos", "<u8"),
                  ("expire_ms", "<i8")])
US_FREE, US_PENDING, US_ACKED, US_REQUEUE, US_DONE = 0, 1, 2, 3, 4
CTRL_TXBUF = 0x80000000     # CtrlRec.seg: data command of a transactional channel (low bits = position)
CTRL_DGET = 0x40000000      # CtrlRec.seg: a Basic.Get its step decoded but could not serve (not paused)

# egress by reference: one gather entry per delivery of a step with Counters.n_ref > 0
# (dp_common.h EgressRef): the len body bytes at host address src go before egress byte dst
EGRESS_REF = np.dtype([("src", "<u8"), ("dst", "<u4"), ("len", "<u4")])

STRUCT_SIZES = {"SegIn": 16, "SegOut": 32, "CtrlRec": 16, "ConnOut": 8, "StepIn": 128, "RDesc": 64, "USlot": 32}
assert RDESC.itemsize == 64

# SegOut.status bits
SS_PAUSED = 1
SS_CTRL = 2
SS_FRAME_ERROR = 4
SS_UNEXPECTED = 8
SS_TOO_LARGE = 16
SS_OVERFLOW = 32

INVALID = 0xFFFFFFFF
U64 = (1 << 64) - 1
FNV64_BASIS = 0xCBF29CE484222325
FNV64_PRIME = 0x100000001B3
GOLDEN64 = 0x9E3779B97F4A7C15


def fnv1a64(data: bytes, h: int = FNV64_BASIS) -> int:
    for b in data:
        h ^= b
        h = (h * FNV64_PRIME) & U64
    return h


def fnv1a32(data: bytes) -> int:
    h = 0x811C9DC5
    for b in data:
        h ^= b
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h


def exch_hash(vhost_id: int, name: bytes) -> int:
    """Device key of an exchange (dataplane.hip exch_hash)."""
    return fnv1a64(name, FNV64_BASIS ^ ((vhost_id * GOLDEN64) & U64))


def direct_key(keyhash: int, exch_slot: int) -> int:
    return keyhash ^ ((exch_slot * GOLDEN64) & U64)


def chan_hash(ch: int) -> int:
    return ((ch * 0x9E3779B1) & 0xFFFFFFFF) >> 7


def split_words_bytes(key: bytes):
    """Java split semantics on bytes (mirror of models.matcher.split_words)."""
    if key == b"":
        return [b""]
    parts = key.split(b".")
    while parts and parts[-1] == b"":
        parts.pop()
    return parts


def topic_pattern_row(pattern: bytes, hash_wildcard=True, nwords_max=8):
    """(int8[256] pattern vector, expect score, flags) for the MFMA topic prefilter."""
    words = split_words_bytes(pattern)
    row = np.zeros(nwords_max * 32, dtype=np.int8)
    dp_only = len(words) > nwords_max or (hash_wildcard and b"#" in words)
    if dp_only:
        return row, -1, 1 | (len(words) << 8)
    nonstar = 0
    star = 0
    for i, w in enumerate(words):
        if w == b"*":
            star |= 1 << i
            continue
        h = fnv1a32(w)
        bits = (h >> np.arange(32, dtype=np.uint64)) & 1
        row[i * 32:(i + 1) * 32] = np.where(bits == 1, 1, -1).astype(np.int8)
        nonstar += 1
    return row, 32 * nonstar, (len(words) << 8) | (star << 16)


def topic_word_offsets(pattern: bytes, nwords_max=8):
    """uint16[8]: (offset << 8 | length) of each pattern word (device exact check)."""
    out = np.zeros(nwords_max, np.uint16)
    words = split_words_bytes(pattern)
    off = 0
    for i, w in enumerate(words[:nwords_max]):
        out[i] = (off << 8) | (len(w) & 255)
        off += len(w) + 1
    return out
