"""Launcher for a sharded broker node: hosts the rendezvous store itself and starts one
process per GPU.

torchrun tears the whole job down when one worker dies and its store may live in a
worker; a broker must keep serving when a rank fails (parallel/node.py failover), so the
store is hosted here — outside every rank — and a rank's exit is reported, not fatal.
Ranks join with ``join()`` (``torch.distributed.init_process_group`` over that store).
"""

import datetime
import os
import subprocess
import sys
import time

import torch.distributed as dist

ENV_STORE = "CHANAMQ_STORE"   # host:port of the launcher's TCPStore


def join(backend="gloo", timeout_s=60):
    """Called inside a rank: init the default process group over the launcher's store.
    Returns (rank, world, store)."""
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    host, port = os.environ[ENV_STORE].rsplit(":", 1)
    store = dist.TCPStore(host, int(port), world_size=world + 1, is_master=False,
                          timeout=datetime.timedelta(seconds=timeout_s), wait_for_workers=False)
    kw = {}
    if backend == "nccl":
        # a peer that dies mid-collective must surface as an exception in this rank's
        # step (Comm._wait -> ShardedNode.handle_failure), not as the RCCL watchdog
        # tearing the process down: no async error handling, bounded blocking waits
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")
        import torch
        local = int(os.environ.get("LOCAL_RANK", rank)) % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        kw["device_id"] = torch.device("cuda", local)
    dist.init_process_group(backend, store=store, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank, world, store


class Launcher:
    def __init__(self, world, argv, host="127.0.0.1", env=None):
        self.world, self.argv = world, list(argv)
        self.store = dist.TCPStore(host, 0, world_size=world + 1, is_master=True,
                                   timeout=datetime.timedelta(seconds=120), wait_for_workers=False)
        self.addr = f"{host}:{self.store.port}"
        self.env = dict(os.environ if env is None else env)
        self.procs = []

    def start(self):
        for r in range(self.world):
            env = dict(self.env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(self.world),
                       **{ENV_STORE: self.addr})
            self.procs.append(subprocess.Popen([sys.executable] + self.argv, env=env))
        return self

    def poll(self):
        """{rank: exit code} of the ranks that have exited."""
        return {r: p.returncode for r, p in enumerate(self.procs) if p.poll() is not None}

    def wait(self, timeout=None):
        end = None if timeout is None else time.time() + timeout
        for p in self.procs:
            p.wait(None if end is None else max(0.1, end - time.time()))
        return [p.returncode for p in self.procs]

    def stop(self, sig=None, timeout=30):
        for p in self.procs:
            if p.poll() is None:
                p.terminate() if sig is None else p.send_signal(sig)
        return self.wait(timeout)


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(prog="chanamq_amd.parallel.launch",
                                 description="start N ranks of a sharded broker: launch N -- script args...")
    ap.add_argument("world", type=int)
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    rest = a.rest[1:] if a.rest[:1] == ["--"] else a.rest
    ln = Launcher(a.world, rest).start()
    codes = ln.wait()
    return max(codes) if codes else 0


if __name__ == "__main__":
    sys.exit(main())
