"""Cold store segment files (chanamq_amd/store/cold.py): appends never cross a segment,
reads return what was written, fully released segments are unlinked."""

import numpy as np

from chanamq_amd.store import cold
from chanamq_amd.store.cold import ColdStore


def test_put_get_segments_and_gc(tmp_path, monkeypatch):
    monkeypatch.setattr(cold, "SEG_SHIFT", 16)
    monkeypatch.setattr(cold, "SEG", 1 << 16)
    st = ColdStore(str(tmp_path / "c"))
    rng = np.random.default_rng(3)
    bodies = [rng.integers(0, 256, int(n), dtype=np.uint8) for n in rng.integers(1, 9000, 300)]
    offs = st.put_many([memoryview(b) for b in bodies])
    assert len(set(offs)) == len(offs)
    for o, b in zip(offs, bodies):   # none crosses a 64 KiB segment
        assert (o >> 16) == ((o + len(b) - 1) >> 16)
    for o, b in zip(offs[::7], bodies[::7]):
        out = np.zeros(len(b), np.uint8)
        st.get_into(o, memoryview(out))
        assert np.array_equal(out, b)
    nseg = (st.head >> 16) + 1
    live = np.zeros(nseg, np.int64)
    live[nseg - 2] = 5                # one older segment still holds a live body
    assert st.gc(live) == nseg - 2    # all but that one and the segment being appended to
    out = np.zeros(len(bodies[-1]), np.uint8)
    st.get_into(offs[-1], memoryview(out))
    assert np.array_equal(out, bodies[-1])
    st.close()


def test_segment_slots_never_alias_after_wrapping(tmp_path, monkeypatch):
    """store offsets only grow but the device counts live bytes per segment at
    [seg % COLD_SEGS].  A new segment skips every number whose slot an open segment still
    uses, and gc indexes the live array the device's way (no 'seg < len' guard, so
    segments past the first wrap are unlinked too)."""
    monkeypatch.setattr(cold, "SEG_SHIFT", 16)
    monkeypatch.setattr(cold, "SEG", 1 << 16)
    st = ColdStore(str(tmp_path / "c"), slots=4)
    body = memoryview(np.zeros(40000, np.uint8))
    segs = lambda offs: sorted({o >> 16 for o in offs})  # noqa: E731
    assert segs(st.put_many([body] * 4)) == [0, 1, 2, 3]
    live = np.zeros(4, np.int64)
    live[1] = 7                                  # segment 1 keeps a live body
    assert st.gc(live) == 2                      # 0 and 2 go; 3 is being appended to
    # next segments: 4 (slot 0, free), not 5 (slot 1 = live segment 1), then 6 (slot 2)
    assert segs(st.put_many([body] * 2)) == [4, 6]
    assert sorted(st.fds) == [1, 3, 4, 6]
    assert len({s % 4 for s in st.fds}) == len(st.fds)
    live[:] = 0
    assert st.gc(live) == 3                      # past the wrap: 1, 3 and 4 unlinked (6 current)
    assert sorted(st.fds) == [6]
    st.close()
