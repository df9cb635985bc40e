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


def _wire_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sdmi.reducer import BucketReducer
    n = 50_000
    init = torch.randn(n, generator=torch.Generator().manual_seed(7))
    for wire in ("fp32", "bf16"):
        p = torch.nn.Parameter(init.clone())
        opt = torch.optim.Adam([p], lr=1e-3)
        grads = torch.zeros(n)
        red = BucketReducer(grads, None, bucket_bytes=16 << 10, wire=wire)
        for s in range(3):
            g = torch.Generator().manual_seed(1000 * s + rank)
            grads.copy_(torch.randn(n, generator=g) * (1 + s) + torch.sin(p.detach() * (rank + 1)))
            red.reset()
            for upto in (n // 3, 2 * n // 3, n):  # backward-ordered release
                red.ready(upto)
            red.finish()
            p.grad = grads / world  # DDP average
            opt.step()
        out[(wire, rank)] = p.detach().clone()
    dist.destroy_process_group()


def test_bf16_gradient_wire_tracks_fp32_after_three_steps():
    """The optional bf16 wire format of the gradient all-reduce (sdmi.reducer, SDMI_GRAD_WIRE=bf16: half the xGMI
    bytes) against the fp32 wire (the reference's DDP arithmetic, train_ddpm_cond_celebhq_multi_gpu.py:257-263) over
    three Adam steps on two gloo ranks: ranks stay bit-identical to each other, and the parameter update differs from
    the fp32 one by at most 2 % in norm (bf16 rounding of the per-rank gradients and of the partial sums: ~2^-9
    relative per element, amplified where the ranks' gradients cancel)."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_wire_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    init = torch.randn(50_000, generator=torch.Generator().manual_seed(7))
    for wire in ("fp32", "bf16"):
        assert torch.equal(out[(wire, 0)], out[(wire, 1)]), wire
    d32, d16 = out[("fp32", 0)] - init, out[("bf16", 0)] - init
    rel = ((d16 - d32).norm() / d32.norm()).item()
    assert 0 < rel <= 2e-2, rel


def _norm_worker(rank, world, port, wire, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sdmi.reducer import BucketReducer, NormBlocks, CPU_NORM_BLOCK
    numel = 5 * CPU_NORM_BLOCK + 1234
    flat = torch.randn(numel + 4, generator=torch.Generator().manual_seed(300 + rank))  # + the trainer's flag tail
    norm = NormBlocks(numel, "cpu")
    red = BucketReducer(flat, None, bucket_bytes=4, wire=wire, norm=norm)  # rounded up to one norm block per bucket
    assert red.bucket == CPU_NORM_BLOCK
    red.reset()
    for m in (1000, CPU_NORM_BLOCK + 7, 3 * CPU_NORM_BLOCK, numel, numel + 4):
        red.ready(m)
    red.finish()
    whole = NormBlocks(numel, "cpu")
    whole.whole(flat)  # one pass over the all-reduced buffer
    out[rank] = (red.nb, torch.equal(norm.partials, whole.partials), norm.partials.clone())
    dist.destroy_process_group()


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_reducer_norm_pieces_equal_whole_buffer_norm(wire):
    """N > 1 gradient norm (train_ddpm_cond_celebhq_multi_gpu.py:362-365 on the DDP-averaged gradients): the reducer
    computes each bucket's norm blocks right after its all-reduce (buckets are whole blocks), and the block partials
    -- hence the finalised norm, summed in block order -- equal one whole-buffer pass over the all-reduced gradients
    bitwise, on both ranks, for the fp32 and the bf16 wire (where the blocks are of the widened values)."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_norm_worker, args=(world, _free_port(), wire, out), nprocs=world, join=True)
    for r in range(world):
        nb, same, _ = out[r]
        assert nb == 6 and same, (r, nb, same)
    assert torch.equal(out[0][2], out[1][2])


class _StandInRccl:
    """Stand-in for libsdmi's RCCL entry points (CPU protocol test of NativeComm.create): `fail` names the entry point
    that fails on rank `bad`; sdmi_allreduce is an identity (a wrong collective) unless `sum_group` is given, in which
    case it all-reduces through gloo (a correct one)."""

    def __init__(self, rank, bad, fail, sum_group=None):
        self.rank, self.bad, self.fail, self.sum_group = rank, bad, fail, sum_group
        self.destroyed = 0

    def _rc(self, name):
        return 1 if (name == self.fail and self.rank == self.bad) else 0

    def sdmi_comm_load(self, path):
        return self._rc("load")

    def sdmi_comm_unique_id(self, uid):
        uid[0] = 7
        return self._rc("uid")

    def sdmi_comm_init(self, uid, world, rank, h):
        h._obj.value = 1 if self._rc("init") == 0 else 0
        return self._rc("init")

    def sdmi_allreduce(self, h, ptr, n, dt, stream):
        return 0

    def sdmi_comm_destroy(self, h):
        self.destroyed += 1
        return 0


def _comm_worker(rank, world, port, fail, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sdmi import reducer as R
    lib = _StandInRccl(rank, bad=0 if fail == "uid" else world - 1, fail=fail)
    comm = R.NativeComm.create(None, "cpu", lib=lib)
    # the self-check on its own: a correct all-reduce passes on every rank, an identity fails on every rank
    good = R.agree(R.allreduce_selfcheck(lambda b: dist.all_reduce(b), rank, world, "cpu"), None, "cpu")
    bad = R.agree(R.allreduce_selfcheck(lambda b: None, rank, world, "cpu"), None, "cpu")
    out[rank] = (comm is None, good, bad)
    dist.destroy_process_group()


@pytest.mark.parametrize("fail", ["load", "uid", "init", "selfcheck"])
def test_native_comm_fallback_is_collective(fail):
    """the library-communicator decision is taken by all ranks together. A failure on ONE rank (binding
    librccl, rank 0's unique id, the communicator init, or an all-reduce that does not sum) makes EVERY rank fall
    back to torch.distributed -- no rank hangs in a broadcast or an init its peers abandoned, no mix of paths."""
    world = 3
    mgr = mp.Manager()
    out = mgr.dict()
    # (fail == "uid" fails on rank 0 -- the only rank that makes an id; "selfcheck": the stand-in's identity
    # all-reduce is wrong on every rank at world > 1)
    mp.spawn(_comm_worker, args=(world, _free_port(), fail, out), nprocs=world, join=True)
    assert all(out[r] == (True, True, False) for r in range(world)), dict(out)
