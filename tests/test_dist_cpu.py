"""Multi-process (world_size 2, gloo, CPU) checks of the data-parallel gradient path:
the BucketReducer all-reduces a flat gradient buffer in backward-ordered buckets exactly like one
all-reduce of the whole buffer, whatever the order in which prefixes become final, and the
trainer's watermark plan never releases a bucket before every gradient in it is final."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, bucket, marks, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sdmi.reducer import BucketReducer
    g = torch.Generator().manual_seed(100 + rank)
    flat = torch.randn(n, generator=g)
    ref = flat.clone()
    dist.all_reduce(ref)
    red = BucketReducer(flat, None, bucket_bytes=bucket * 4)
    red.reset()
    for m in marks:
        red.ready(m)
    red.finish()
    out[rank] = float((flat - ref).abs().max())
    dist.destroy_process_group()


@pytest.mark.parametrize("marks", [[0, 10, 999, 5000, 10000], [10000], [3, 3, 7000, 9999, 10000]])
def test_bucket_reducer_matches_allreduce(marks):
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), 10000, 1024, marks, out), nprocs=world, join=True)
    assert all(out[r] == 0.0 for r in range(world)), dict(out)


def test_watermarks_respect_labels():
    """Every bucket released at backward position k contains only parameters whose label completed."""
    from oracle import sd_oracle as O
    from tests.golden.configs import full_cond_config
    from sdmi.store import FlatStore, param_label
    from sdmi.trainer import DDPMTrainer
    cfg = full_cond_config()
    shapes = O.unet_param_shapes(cfg)
    st = FlatStore(shapes, cfg, "cpu", with_grads=False)
    # synthetic tape in forward order: input, time, downs, mids, ups, head (what UNetEngine emits)
    labels = ["input", "time"] + [f"downs.{i}" for i in range(3)] * 2 + ["mids.0"] * 3 + \
             [f"ups.{j}" for j in range(3) for _ in range(2)] + ["head"]
    labels = sorted(labels, key=lambda l: ["input", "time", "downs", "mids", "ups", "head"].index(l.split(".")[0]))
    tape = [(None, {"label": l}) for l in labels]
    fake = DDPMTrainer.__new__(DDPMTrainer)
    fake.store = st
    marks = fake._watermarks(tape)
    done = {}
    for k in range(len(tape) - 1, -1, -1):
        done[tape[k][1]["label"]] = k
    for k in range(len(tape) - 1, -1, -1):
        completed = {l for l, kk in done.items() if kk >= k}
        upto = 0
        for end, run in marks:
            if run >= k:
                upto = end
            else:
                break
        for key in st.order:
            off, n = st.offsets[key]
            if off + n <= upto:
                assert param_label(key) in completed, (k, key)
