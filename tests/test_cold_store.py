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
