"""Cold store: the third tier of message bodies, below HBM and the pinned-host spill ring.

The reference keeps message bodies in MessageEntity actors and, once a body has been idle
for ``chana.mq.message.inactive``, writes even a non-persistent one to Cassandra and
passivates the actor; ``Get`` reloads it lazily (chana-mq-server/.../entity/
MessageEntity.scala:82-102,174-186).  Here the device lists cold spilled bodies
(``k_cold_pick``), this store appends them to segment files, and the device then holds a
queue's deliveries at the first cold position until the bodies are read back into the
spill ring (``k_cold_scan`` / ``k_cold_in``): backlog depth is bounded by the disk, not by
HBM or host RAM.

Layout: 1 GiB segment files ``cold-<n>.seg`` (dp_common.h COLD_SEG_SHIFT); a record never
crosses a segment; the device keeps live bytes per segment (``cold_live``) and ``gc``
unlinks segments that are fully released.  Restart semantics: cold bodies are of
non-persistent messages only (persistent ones stay in the WAL store), which a restart
drops anyway, so the store is wiped when it opens.
"""

import os
import shutil
import tempfile

import numpy as np

SEG_SHIFT = 30
SEG = 1 << SEG_SHIFT
SLOTS = 16384      # dp_common.h COLD_SEGS: the device counts segment s's live bytes at [s % SLOTS]
COLD_REC = np.dtype([("msg", "<u4"), ("q", "<u4"), ("qpos", "<u8"), ("pos", "<u8"), ("cold", "<u8"),
                     ("bytes", "<u4"), ("pad", "<u4")])
assert COLD_REC.itemsize == 40


class ColdStore:
    def __init__(self, path=None, slots=SLOTS):
        self.own = path is None
        self.slots = slots
        self.path = path or tempfile.mkdtemp(prefix="cmq-cold-")
        if os.path.isdir(self.path):
            for f in os.listdir(self.path):
                if f.endswith(".seg"):
                    os.unlink(os.path.join(self.path, f))
        os.makedirs(self.path, exist_ok=True)
        self.head = 0           # next free store offset
        self.fds = {}
        self.written = self.read = 0

    def _fd(self, seg):
        fd = self.fds.get(seg)
        if fd is None:
            fd = os.open(os.path.join(self.path, f"cold-{seg}.seg"), os.O_CREAT | os.O_RDWR, 0o600)
            self.fds[seg] = fd
        return fd

    def put_many(self, views):
        """Append the byte views; returns their store offsets (one pwritev per segment run)."""
        offs, batch, bstart = [], [], None
        for v in views:
            n = len(v)
            if (self.head & (SEG - 1)) + n > SEG:        # never across a segment
                self._flush(batch, bstart)
                batch, bstart = [], None
                self.head = self._next_seg(self.head >> SEG_SHIFT) << SEG_SHIFT
            if bstart is None:
                bstart = self.head
            offs.append(self.head)
            batch.append(v)
            self.head += n
            if len(batch) >= 512:
                self._flush(batch, bstart)
                batch, bstart = [], None
        self._flush(batch, bstart)
        return offs

    def _next_seg(self, cur):
        """The segment after ``cur`` whose live-byte slot (seg % slots) no open segment
        uses: offsets grow without bound, slots wrap, and two live segments must never
        share one (the device's count would mix them and gc could unlink a live one)."""
        used = {seg % self.slots for seg in self.fds}
        seg = cur + 1
        for _ in range(self.slots):
            if seg % self.slots not in used:
                return seg
            seg += 1
        raise OSError("cold store: every segment slot holds live bodies")

    def _flush(self, batch, start):
        if not batch:
            return
        fd = self._fd(start >> SEG_SHIFT)
        want = sum(len(v) for v in batch)
        done = os.pwritev(fd, batch, start & (SEG - 1))
        if done != want:
            raise OSError(f"cold store: short write ({done} of {want} bytes)")
        self.written += want

    def get_into(self, off, dst):
        fd = self._fd(off >> SEG_SHIFT)
        n = os.preadv(fd, [dst], off & (SEG - 1))
        if n != len(dst):
            raise OSError(f"cold store: short read at {off} ({n} of {len(dst)} bytes)")
        self.read += n

    def gc(self, live):
        """Unlink the segments the device reports fully released (``live``: int64 per
        segment), except the one being appended to."""
        cur = self.head >> SEG_SHIFT
        n = 0
        for seg in list(self.fds):   # (slots never alias: _next_seg)
            if seg != cur and live[seg % len(live)] <= 0:
                os.close(self.fds.pop(seg))
                os.unlink(os.path.join(self.path, f"cold-{seg}.seg"))
                n += 1
        return n

    def bytes_on_disk(self):
        return sum(os.fstat(fd).st_size for fd in self.fds.values())

    def close(self):
        for fd in self.fds.values():
            os.close(fd)
        self.fds = {}
        if self.own:
            shutil.rmtree(self.path, ignore_errors=True)
