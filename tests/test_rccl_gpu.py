"""RCCL on the one-GPU box: an "nccl" process group (RCCL over xGMI on ROCm) of world size 1, the trainer's
BucketReducer forced on, the step recorded once by sdmi.plan.StepPlan and replayed. The bucket all-reduces run
through RCCL on the reducer stream between the backward's gradient producers and the optimizer; with one rank
they are identities, so parameters, Adam moments, EMA and GradScaler state must be bit-identical to a trainer
without a reducer fed the same inputs. Both issue paths: the library's own RCCL communicator (native plan ops,
csrc/comm.hip) and torch.distributed callouts (SDMI_NATIVE_COMM=0)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(step, B=2):
    g = torch.Generator().manual_seed(900 + step)
    x0 = torch.randn(B, 4, 32, 32, generator=g)
    noise = torch.randn(B, 4, 32, 32, generator=g)
    t = torch.randint(0, 1000, (B,), generator=g)
    text = torch.randn(B, 77, 64, generator=g)
    cmap = torch.randint(0, 19, (B, 64, 64), generator=g)
    mask = torch.nn.functional.one_hot(cmap, 19).movedim(-1, 1)[:, 1:].float()
    return [v.cuda() for v in (x0, noise, t, text, mask)]


def _worker(rank, port, out, native):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SDMI_NATIVE_COMM=native)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from oracle import sd_oracle as O
    from tests.golden.configs import SMALL_COND
    from sdmi.trainer import DDPMTrainer
    from sdmi.plan import StepPlan
    sd = O.deterministic_state(O.unet_param_shapes(SMALL_COND), seed=3)
    red = DDPMTrainer(SMALL_COND, sd, "cuda", lr=1e-3, group=dist.group.WORLD, force_reducer=True,
                      bucket_bytes=1 << 20)
    assert red.reducer is not None and red.world == 1
    assert (red.reducer.comm is not None) == (native == "1")
    ref = DDPMTrainer(SMALL_COND, sd, "cuda", lr=1e-3)
    bufs = [torch.empty_like(v) for v in _inputs(0)]
    plan = None
    for s in range(4):
        for b, v in zip(bufs, _inputs(s)):
            b.copy_(v)
        ref.step(*bufs)
        if plan is None:
            plan = StepPlan(lambda: red.step(*bufs))
        else:
            plan.replay()
    red.sync_optimizer()
    ref.sync_optimizer()
    torch.cuda.synchronize()
    ok = (torch.equal(red.store.params, ref.store.params) and torch.equal(red.m, ref.m)
          and torch.equal(red.v, ref.v) and torch.equal(red.ema, ref.ema) and torch.equal(red.state, ref.state))
    out["ok"] = ok
    out["collectives"] = plan.collectives()
    out["reducer_callouts"] = sum(1 for fn, _ in plan.ops if getattr(fn, "__name__", "") in ("_issue", "_wait"))
    out["backend"] = dist.get_backend()
    dist.destroy_process_group()


@pytest.mark.parametrize("native", ["1", "0"])
def test_rccl_bucket_allreduce_in_replayed_plan(native):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(_port(), out, native), nprocs=1, join=True)
    assert out["backend"] == "nccl"
    assert out["collectives"] >= 2  # the flat gradient buffer went out in more than one bucket
    if native == "1":
        assert out["reducer_callouts"] == 0  # the exchange replays natively
    assert out["ok"]


def _wire_worker(rank, port, out):
    """bf16 gradient wire through RCCL, both issue paths: one rank makes the all-reduce an identity, so the library's
    communicator (ncclBfloat16) and torch.distributed must leave bitwise the same trainer state."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from oracle import sd_oracle as O
    from tests.golden.configs import SMALL_COND
    from sdmi.trainer import DDPMTrainer
    sd = O.deterministic_state(O.unet_param_shapes(SMALL_COND), seed=4)
    trs = {}
    for native in ("1", "0"):
        os.environ["SDMI_NATIVE_COMM"] = native
        trs[native] = DDPMTrainer(SMALL_COND, sd, "cuda", lr=1e-3, group=dist.group.WORLD, force_reducer=True,
                                  bucket_bytes=1 << 20, grad_wire="bf16")
    assert trs["1"].reducer.comm is not None and trs["0"].reducer.comm is None
    for s in range(3):
        inp = _inputs(s)
        for tr in trs.values():
            tr.step(*inp)
    for tr in trs.values():
        tr.sync_optimizer()
    torch.cuda.synchronize()
    a, b = trs["1"], trs["0"]
    out["ok"] = (torch.equal(a.store.params, b.store.params) and torch.equal(a.m, b.m) and torch.equal(a.v, b.v)
                 and torch.equal(a.state, b.state))
    dist.destroy_process_group()


def test_rccl_bf16_wire_native_matches_torch_distributed():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_wire_worker, args=(_port(), out), nprocs=1, join=True)
    assert out["ok"]


def _dit_worker(rank, port, out):
    """The DiT trainer (one weight-gradient stream, no context stream: the reducer takes a stream of its own) with the
    bucket reducer forced on over the library's RCCL communicator, recorded once and replayed: bit-identical to the
    reducer-free DiT trainer fed the same inputs."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SDMI_NATIVE_COMM="1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from oracle import sd_oracle as O, dit_oracle as DO
    from tests.golden.configs import SMALL_DIT
    from sdmi.trainer import DDPMTrainer
    from sdmi.plan import StepPlan
    sd = O.deterministic_state(DO.dit_param_shapes(SMALL_DIT), seed=5)
    red = DDPMTrainer(SMALL_DIT, sd, "cuda", base="dit", lr=1e-3, ema_decay=None, group=dist.group.WORLD,
                      force_reducer=True, bucket_bytes=1 << 18)
    assert red.reducer is not None and red.reducer.comm is not None
    ref = DDPMTrainer(SMALL_DIT, sd, "cuda", base="dit", lr=1e-3, ema_decay=None)
    bufs = [torch.empty_like(v) for v in _inputs(0)]
    plan = None
    for s in range(4):
        for b, v in zip(bufs, _inputs(s)):
            b.copy_(v)
        ref.step(*bufs)
        if plan is None:
            plan = StepPlan(lambda: red.step(*bufs))
        else:
            plan.replay()
    red.sync_optimizer()
    ref.sync_optimizer()
    torch.cuda.synchronize()
    out["ok"] = (torch.equal(red.store.params, ref.store.params) and torch.equal(red.m, ref.m)
                 and torch.equal(red.v, ref.v) and torch.equal(red.state, ref.state))
    out["collectives"] = plan.collectives()
    dist.destroy_process_group()


def test_rccl_dit_reducer_in_replayed_plan():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_dit_worker, args=(_port(), out), nprocs=1, join=True)
    assert out["collectives"] >= 2
    assert out["ok"]
