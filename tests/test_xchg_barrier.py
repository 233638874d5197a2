"""The shared-memory exchange's barrier agrees on its outcome (xchg_host.h).

A rank that times out withdraws its arrival, so a late peer cannot complete the
generation behind its back: either every member passes, or every member reports -2
and drops the step's exchange together; the barrier stays usable afterwards."""

import multiprocessing as mp
import os
import time


def _member(name, me, delay, q):
    from chanamq_amd.broker import load
    core = load()
    x = core.ShmXchg(name, [0, 1], me, 4096, 300)
    out = []
    time.sleep(delay)
    out.append(x.barrier())          # rank 1 comes 0.8 s late: both must time out
    time.sleep(1.0 - delay)          # re-align (rank 0 has been back for a while)
    out.append(x.barrier())          # both on time: both pass
    out.append(x.barrier())
    q.put((me, out))


def test_late_member_cannot_split_the_outcome():
    name = f"cmq_bar_{os.getpid()}"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_member, args=(name, 0, 0.0, q)),
          ctx.Process(target=_member, args=(name, 1, 0.8, q))]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=60) for _ in ps)
    for p in ps:
        p.join(30)
    try:
        os.unlink("/dev/shm/" + name)
    except FileNotFoundError:
        pass
    assert res[0][0] == res[1][0] == -2, res
    assert res[0][1:] == res[1][1:] == [0, 0], res


def _member_eager(name, me, delay, n_calls, q):
    from chanamq_amd.broker import load
    core = load()
    x = core.ShmXchg(name, [0, 1], me, 4096, 300)
    time.sleep(delay)
    q.put((me, [x.barrier() for _ in range(n_calls)]))


def test_withdrawn_member_reentering_at_once_never_pairs_with_a_late_peer():
    """a rank that timed out calls the barrier again right away (the control
    plane resumed it) while its peer is still on its way to the generation the rank just
    failed.  Arrivals carry their generation, so the early rank's next arrival aborts the
    failed generation instead of completing it for the late peer: generation by generation
    (= call by call) both ranks report the same outcome, whatever the timing, and once the
    late rank has caught up they pass together."""
    ctx = mp.get_context("spawn")
    for k, delay in enumerate((0.45, 0.75, 1.05)):
        name = f"cmq_bar2_{os.getpid()}_{k}"
        q = ctx.Queue()
        ps = [ctx.Process(target=_member_eager, args=(name, 0, 0.0, 6, q)),
              ctx.Process(target=_member_eager, args=(name, 1, delay, 6, q))]
        for p in ps:
            p.start()
        res = dict(q.get(timeout=60) for _ in ps)
        for p in ps:
            p.join(30)
        try:
            os.unlink("/dev/shm/" + name)
        except FileNotFoundError:
            pass
        assert res[0] == res[1], (delay, res)
        assert res[0][0] == -2 and res[0][-1] == 0, (delay, res)
