"""Small-table engine config shared by the GPU tests (fits any test scenario)."""
CFG = dict(c_max=64, chpc=8, q_max=64, x_max=64, cons_max=256, seg_max=64, cmd_max=4096, deliv_max=4096,
           msg_max=1 << 14, ucap=256, deliver_cap=4096, ingress_cap=8 << 20, egress_cap=16 << 20,
           log_bytes=64 << 20, log_block=1 << 20, ring_pool=1 << 20, default_queue_capacity=1 << 12, tb_max=64,
           carry_cap=1 << 18, dhash=1024, req_max=4096)
