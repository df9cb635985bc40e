"""Data-parallel trainer on the GPU: two ranks share cuda:0 through the gloo backend (the box has one
GPU; RCCL needs distinct devices). Checks that the bucketed, backward-overlapped all-reduce of
sdmi.trainer gives the same update as one process that averages the two ranks' gradients:
parameters after one step agree to fp32 rounding of the averaging order."""
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


def _batch(rank, cfg):
    g = torch.Generator().manual_seed(50 + rank)
    B = 2
    x0 = torch.randn(B, 4, 32, 32, generator=g)
    noise = torch.randn(B, 4, 32, 32, generator=g)
    t = torch.randint(0, 1000, (B,), generator=g)
    text = torch.randn(B, 77, 64, generator=g)
    cmap = torch.randint(0, 19, (B, 64, 64), generator=g)
    mask = torch.nn.functional.one_hot(cmap, 19).movedim(-1, 1)[:, 1:].float()
    return [v.cuda() for v in (x0, noise, t, text, mask)]


def _init_state(cfg):
    from oracle import sd_oracle as O
    return O.deterministic_state(O.unet_param_shapes(cfg), seed=1)


def _dit_state():
    from oracle import sd_oracle as O, dit_oracle as DO
    from tests.golden.configs import SMALL_DIT
    return O.deterministic_state(DO.dit_param_shapes(SMALL_DIT), seed=1)


def _worker(rank, world, port, out, model="unet"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests.golden.configs import SMALL_COND, SMALL_DIT
    from sdmi.trainer import DDPMTrainer
    if model == "dit":
        tr = DDPMTrainer(SMALL_DIT, _dit_state(), "cuda", base="dit", lr=1e-3, ema_decay=None,
                         group=dist.group.WORLD, bucket_bytes=1 << 18)
    else:
        tr = DDPMTrainer(SMALL_COND, _init_state(SMALL_COND), "cuda", lr=1e-3, group=dist.group.WORLD,
                         bucket_bytes=1 << 20)
    x0, noise, t, text, mask = _batch(rank, SMALL_COND)
    tr.step(x0, noise, t, text, mask)
    torch.cuda.synchronize()
    if rank == 0:
        out["params"] = tr.store.params.cpu()
        out["norm"] = tr.state[0].item()
    dist.destroy_process_group()


def test_two_rank_step_matches_grad_average():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _port(), out), nprocs=world, join=True)
    # single process: average the two ranks' gradients by hand, same optimizer
    from tests.golden.configs import SMALL_COND
    from sdmi.trainer import DDPMTrainer
    from sdmi import _lib, kernels as K
    tr = DDPMTrainer(SMALL_COND, _init_state(SMALL_COND), "cuda", lr=1e-3)
    gsum = torch.zeros_like(tr.store.grads)
    for r in range(world):
        x0, noise, t, text, mask = _batch(r, SMALL_COND)
        xt = torch.empty_like(x0)
        K.add_noise(x0, noise, t, tr.sqrt_abar, tr.sqrt_1m_abar, xt)
        pred, ctx = tr.engine.forward(xt, t, text, mask)
        dpred = torch.empty(2 * 1024, 8, dtype=torch.bfloat16, device="cuda")
        K.mse(pred, 8, noise, 2, 4, 1024, 1.0, dpred, tr.state[6:7], gscale_dev=tr.state[2:3])
        tr.engine.backward(ctx, dpred)
        gsum += tr.store.grads
    tr.store.grads.copy_(gsum)
    L = _lib.lib()
    ws = torch.empty(L.sdmi_optim_workspace() // 4, device="cuda")
    _lib.check(L.sdmi_clip_unscale(tr.store.grads.data_ptr(), tr.store.numel, 1.0, tr.state.data_ptr(), ws.data_ptr(),
                                   2000, 1, 2.0, K._stream()), "clip")
    _lib.check(L.sdmi_adam_ema(tr.store.params.data_ptr(), tr.store.grads.data_ptr(), tr.m.data_ptr(), tr.v.data_ptr(),
                               tr.ema.data_ptr(), tr.store.numel, tr.state.data_ptr(), 1e-3, 0.9, 0.999, 1e-8, 0.9999,
                               K._stream()), "adam")
    torch.cuda.synchronize()
    assert abs(tr.state[0].item() - out["norm"]) <= 1e-4 * out["norm"]
    diff = (tr.store.params.cpu() - out["params"]).abs().max().item()
    assert diff <= 1e-6, diff


def test_two_rank_dit_step_matches_grad_average():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _port(), out, "dit"), nprocs=world, join=True)
    from tests.golden.configs import SMALL_DIT, SMALL_COND
    from sdmi.trainer import DDPMTrainer
    from sdmi import _lib, kernels as K
    tr = DDPMTrainer(SMALL_DIT, _dit_state(), "cuda", base="dit", lr=1e-3, ema_decay=None)
    gsum = torch.zeros_like(tr.store.grads)
    for r in range(world):
        x0, noise, t, text, mask = _batch(r, SMALL_COND)
        xt = torch.empty_like(x0)
        K.add_noise(x0, noise, t, tr.sqrt_abar, tr.sqrt_1m_abar, xt)
        pred, ctx = tr.engine.forward(xt, t, text, mask)
        dpred = tr.engine.new_dpred(2, 32, 32)
        tr.engine.loss(pred, noise, dpred, tr.state[6:7], gscale_dev=tr.state[2:3])
        tr.engine.backward(ctx, dpred)
        gsum += tr.store.grads
    tr.store.grads.copy_(gsum)
    L = _lib.lib()
    ws = torch.empty(L.sdmi_optim_workspace() // 4, device="cuda")
    _lib.check(L.sdmi_clip_unscale(tr.store.grads.data_ptr(), tr.store.numel, 1.0, tr.state.data_ptr(), ws.data_ptr(),
                                   2000, 1, 2.0, K._stream()), "clip")
    _lib.check(L.sdmi_adam_ema(tr.store.params.data_ptr(), tr.store.grads.data_ptr(), tr.m.data_ptr(), tr.v.data_ptr(),
                               None, tr.store.numel, tr.state.data_ptr(), 1e-3, 0.9, 0.999, 1e-8, 0.0,
                               K._stream()), "adam")
    torch.cuda.synchronize()
    assert abs(tr.state[0].item() - out["norm"]) <= 1e-4 * out["norm"]
    diff = (tr.store.params.cpu() - out["params"]).abs().max().item()
    assert diff <= 1e-6, diff
