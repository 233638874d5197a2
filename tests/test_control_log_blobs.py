"""Control-log bulk payloads (ControlLog.submit(blob=..., blob_to=...)): a replicated op
whose bytes travel only to the named ranks through one variable-size all-to-all at the
sync, not inside the all-gathered JSON (sharded large publishes use it).  Three gloo
ranks on the CPU."""

import multiprocessing as mp
import os

from test_sharded_golden import _free_port


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    import torch.distributed as dist

    from chanamq_amd.parallel.comm import Comm
    from chanamq_amd.parallel.control_log import ControlLog
    dist.init_process_group("gloo")
    log = ControlLog(plane=None, comm=Comm(timeout_s=20))
    seen = []
    log.handlers["big_publish"] = lambda tag, blob=None: seen.append((tag, None if blob is None else len(blob),
                                                                      blob[:4] if blob else None))
    # rank 1 ships 3 MB to ranks 0 and 2; rank 2 ships to itself; rank 0 sends a blob-less op
    if rank == 1:
        log.submit("big_publish", "a", blob=b"AAAA" + os.urandom(3 << 20), blob_to=[0, 2])
        log.submit("big_publish", "b", blob=b"BBBB" * 10, blob_to=[2])
    if rank == 2:
        log.submit("big_publish", "c", blob=b"CCCC", blob_to=[2])
    if rank == 0:
        log.submit("big_publish", "d")
    log.sync()
    log.sync()          # an empty sync afterwards: no all-to-all, nothing applied
    q.put((rank, seen))
    dist.destroy_process_group()


def test_blobs_reach_only_their_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    # applied in (rank, seq) order everywhere
    assert res[0] == [("d", None, None), ("a", (3 << 20) + 4, b"AAAA"), ("b", None, None), ("c", None, None)]
    assert res[1] == [("d", None, None), ("a", None, None), ("b", None, None), ("c", None, None)]
    assert res[2] == [("d", None, None), ("a", (3 << 20) + 4, b"AAAA"), ("b", 40, b"BBBB"), ("c", 4, b"CCCC")]
