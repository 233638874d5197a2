import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import bench
from chanamq_amd.engine.dataplane import GpuDataPlane
P, Q = 256, 16
cfg = dict(c_max=1024, chpc=4, q_max=64, cons_max=1024, seg_max=1024, cmd_max=1 << 17, deliv_max=1 << 16,
           msg_max=1 << 22, ucap=4096, deliver_cap=8192, ingress_cap=64 << 20, egress_cap=128 << 20,
           log_bytes=16 << 30, ring_pool=Q * 2 * (1 << 20), tb_max=64, carry_cap=256 << 10, fs_marks=1)
dp = GpuDataPlane(**cfg)
pool, segs, offs, blens, mps, mb, _ = bench.build_workload(dp, 0, P, Q, 1024, 65536, 8, cons_base=P)
for s in range(6):
    r = dp.step_raw(segs[s % 8], pool.ctypes.data + offs[s % 8], blens[s % 8])
dbg = np.frombuffer(dp.eng.download("dbg", 0, 8 * 16 * 1024), np.uint64).reshape(1024, 16)[:P].astype(np.int64)
ph = np.diff(dbg[:, :9], axis=1) / 100.0  # us
print("phase us (median / max over segments):")
for k in range(8):
    print(k, f"{np.median(ph[:, k]):8.1f} {ph[:, k].max():8.1f}")
print("total", np.median(dbg[:, 8] - dbg[:, 0]) / 100, (dbg[:, 8] - dbg[:, 0]).max() / 100)
sub = [(15, 0, "segment copy (carry + ingress -> work)"), (0, 12, "a: screen + LDS stage"), (12, 13, "a: raw count + scan"), (13, 14, "a: compaction"),
       (14, 1, "a: validation + tail"), (2, 9, "c: (b) tails + sync"), (9, 10, "c: fail compaction"), (10, 11, "c: walk"), (11, 3, "c: expand")]
for a, b, name in sub:
    print(name, f"{np.median(dbg[:, b] - dbg[:, a]) / 100:8.2f}")
print("block start spread us", (dbg[:, 0].max() - dbg[:, 0].min()) / 100)
