"""One rank of the CPU rehearsal of the sharded front end (tests/test_frontend_sharded.py):
EchoEngine(world, rank) + Frontend, the lockstep stepper over the shared-memory exchange.
Control commands ("CTRL") request a control sync; at FE_SYNC every connection gets
"SYNC<step>;" and at FE_XFAIL the rank rebuilds its exchange over itself and reports
"FAILOVER<step>;"."""

import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from chanamq_amd.broker import load  # noqa: E402

FE_OPEN, FE_CLOSED, FE_HOST, FE_CTRL, FE_SYNC, FE_XFAIL = 1, 2, 3, 4, 11, 12


def main():
    rank, world, name, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    async_x = len(sys.argv) > 5 and sys.argv[5] == "async"
    core = load()
    eng = core.EchoEngine(c_max=64, seg_max=64, ingress_cap=1 << 20, carry_cap=1 << 16, world=world, rank=rank)
    eng.xchg_setup(name, list(range(world)), 2000, async_x)
    fe = core.Frontend(eng.c_api(), {"io_threads": 2, "idle_step_ms": 1.0, "per_conn_read": 4096})
    fe.start()
    with open(out + ".tmp", "w") as f:
        f.write(str(fe.port))
    os.replace(out + ".tmp", out)
    conns, waiting, chain = set(), [], 0
    deadline = time.time() + 120
    while time.time() < deadline and not os.path.exists(out + ".stop"):
        for kind, conn, a, b, data, data2 in fe.poll_events(20):
            if kind == FE_OPEN:
                conns.add(conn)
                fe.set_data_mode(conn, b"")
            elif kind == FE_CLOSED:
                conns.discard(conn)
                fe.close(conn)
            elif kind == FE_CTRL:
                waiting.append(conn)
                chain = 1       # a second sync requested while the first is handled
                fe.request_sync()
            elif kind in (FE_SYNC, FE_XFAIL):
                if kind == FE_XFAIL:   # the peer is gone: this rank goes on alone
                    eng.xchg_setup(name + f"-e1r{rank}", [rank], 2000, async_x)
                tag = b"SYNC" if kind == FE_SYNC else b"FAILOVER"
                for c in sorted(conns):
                    fe.send(c, tag + str(a).encode() + b";")
                if kind == FE_SYNC and chain:
                    chain -= 1
                    fe.request_sync()
                for c in waiting:
                    eng.unpause(c)
                    fe.kick(c)
                waiting = []
                fe.sync_done()
    fe.stop()
    st = fe.stats()
    print(f"rank {rank}: steps {st['steps']} xchg {st['xchg_steps']} syncs {st['syncs']} xfails {st['xfails']} "
          f"imported {eng.imported} xchg_us_per_step {1e6 * st['xchg_s'] / max(1, st['xchg_steps']):.1f}", flush=True)
    with open(out + ".stats", "w") as f:
        f.write(f"{st['xchg_s']} {st['xchg_steps']} {st['syncs']} {st['xfails']}")


if __name__ == "__main__":
    main()
