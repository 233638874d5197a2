"""Diagnose a control reply that never arrives on the pipelined GPU server: the confirmed
publish scenario of tests/test_gpu_broker.py, then a new connection's Channel.Open; on a
timeout, dump the control-plane / stepper state (held replies, submitted / finished steps,
staged table writes, lock state) twice a second apart."""
import sys
import os
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def dump(b, tag):
    fe, lk = b.fe, b.lock
    print(tag, "ctl_state", fe.ctl_state(), "steps", fe.stats()["steps"], "deltas", b.plane.eng.deltas_pending(),
          "lock depth", lk.depth, "paused_at", lk.paused_at, "light", lk.light, "defer", b.plane.defer,
          "conns", {k: v.state for k, v in b.conns.items()}, flush=True)


def main():
    from test_gpu_broker import GPU_CFG
    from chanamq_amd.client import Connection
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.server.gpu_broker import GpuBroker
    for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        b = GpuBroker(GpuDataPlane(default_queue_capacity=1 << 12, **GPU_CFG), idle_step_ms=1.0, io="pipeline",
                      ingress_bytes=8 << 20).start()
        try:
            p = Connection(port=b.port, vhost="/")
            ch = p.channel()
            ch.queue_declare("deep")
            ch.confirm_select()
            for i in range(12000):
                ch.basic_publish("", "deep", i.to_bytes(4, "big"))
                if i % 2000 == 1999:
                    p.process(0.01)
            assert ch.wait_for_confirms(timeout=60)
            assert ch.queue_declare("deep", passive=True).message_count == 12000
            c = Connection(port=b.port, vhost="/", timeout=5)
            try:
                c.channel()
                print("rep", rep, "ok", flush=True)
            except Exception as e:
                print("rep", rep, "FAILED", repr(e), flush=True)
                dump(b, "t0")
                time.sleep(1.0)
                dump(b, "t1")
                return 1
            p.close()
            c.close()
        finally:
            b.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
