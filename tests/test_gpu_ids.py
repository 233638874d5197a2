"""Snowflake ids (K13) on the HIP plane: 64 worker ids per GPU keep the virtual position
behind the wall clock, and recovery seeds new ids above every stored one."""

import time

import pytest

from gpu_cfg import CFG

pytestmark = pytest.mark.gpu

VH = "AMQ.DEFAULT"


def _plane():
    from chanamq_amd.engine.dataplane import GpuDataPlane
    return GpuDataPlane(persist=1, persist_max=4096, persist_bytes=8 << 20, restore_max=1024,
                        restore_bytes=8 << 20, **CFG)


def _publish(plane, pers, n, tag):
    from chanamq_amd.engine.traffic import publish_command
    data = b"".join(publish_command(1, "", "ids.q", b"%s-%d" % (tag, i), {"delivery_mode": 2}) for i in range(n))
    plane.step({1: data})
    pers.after_step()
    pers.commit()


def test_ids_fit_the_wall_clock_and_survive_restart(gpu, tmp_path):
    from chanamq_amd.broker import load
    from chanamq_amd.engine.persistence import GpuPersistence
    core = load()
    st = core.Store()
    st.open(str(tmp_path / "s"), True)
    p1 = _plane()
    pers = GpuPersistence(p1, st)
    p1.declare_queue(VH, "ids.q", durable=True)
    pers.queue(p1.queues[(VH, "ids.q")])
    p1.open_connection(1, VH)
    p1.open_channel(1, 1)
    t0 = int(time.time() * 1000)
    _publish(p1, pers, 2000, b"a")                  # 2000 ids in one step (6000 frames < CAND_MAX)
    ids1 = sorted(st.message_ids())
    assert len(ids1) == 2000 and len(set(ids1)) == 2000
    ms = {i >> 22 for i in ids1}
    assert max(ms) <= int(time.time() * 1000) + 1 and min(ms) >= t0 - 1   # no virtual-clock drift
    workers = {(i >> 12) & 1023 for i in ids1}
    assert workers <= set(range(64))                # rank 0 owns worker ids 0..63
    # the device clock ran far ahead before a crash (e.g. a clock step back afterwards)
    p1.seed_ids(t0 + 60_000)
    _publish(p1, pers, 10, b"b")
    ahead = [i for i in st.message_ids() if (i >> 22) >= t0 + 60_000]
    assert len(ahead) == 10
    del p1
    st.close()

    st2 = core.Store()
    st2.open(str(tmp_path / "s"), True)
    p2 = _plane()
    pers2 = GpuPersistence(p2, st2)
    assert pers2.recover(int(time.time() * 1000)) == 2010
    old = set(st2.message_ids())
    p2.open_connection(1, VH)
    p2.open_channel(1, 1)
    _publish(p2, pers2, 50, b"c")
    new = set(st2.message_ids()) - old
    assert len(new) == 50
    assert min(new) > max(old)                      # seeded above every recovered id
    st2.close()
