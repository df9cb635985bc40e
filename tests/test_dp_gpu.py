"""Data-parallel trainer on the GPU: two ranks share cuda:0 through the gloo backend (the box has one
GPU; RCCL needs distinct devices). Checks that the bucketed, backward-overlapped all-reduce of
sdmi.trainer gives the same update as one process that averages the two ranks' gradients:
parameters after three steps agree to fp32 rounding of the averaging order. The ranks start from DIFFERENT
weights: the trainer must broadcast rank 0's (as DDP does at wrap time), so rank 1's own init is discarded."""
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


STEPS = 3


def _batch(rank, cfg, step=0):
    g = torch.Generator().manual_seed(50 + rank + 100 * step)
    B = 2
    x0 = torch.randn(B, 4, 32, 32, generator=g)
    noise = torch.randn(B, 4, 32, 32, generator=g)
    t = torch.randint(0, 1000, (B,), generator=g)
    text = torch.randn(B, 77, 64, generator=g)
    cmap = torch.randint(0, 19, (B, 64, 64), generator=g)
    mask = torch.nn.functional.one_hot(cmap, 19).movedim(-1, 1)[:, 1:].float()
    return [v.cuda() for v in (x0, noise, t, text, mask)]


def _init_state(cfg, rank=0):
    from oracle import sd_oracle as O
    return O.deterministic_state(O.unet_param_shapes(cfg), seed=1 + rank)


def _dit_state(rank=0):
    from oracle import sd_oracle as O, dit_oracle as DO
    from tests.golden.configs import SMALL_DIT
    return O.deterministic_state(DO.dit_param_shapes(SMALL_DIT), seed=1 + rank)


def _worker(rank, world, port, out, model="unet"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests.golden.configs import SMALL_COND, SMALL_DIT
    from sdmi.trainer import DDPMTrainer
    if model == "dit":
        tr = DDPMTrainer(SMALL_DIT, _dit_state(rank), "cuda", base="dit", lr=1e-3, ema_decay=None,
                         group=dist.group.WORLD, bucket_bytes=1 << 18)
    else:
        tr = DDPMTrainer(SMALL_COND, _init_state(SMALL_COND, rank), "cuda", lr=1e-3, group=dist.group.WORLD,
                         bucket_bytes=1 << 20)
    for s in range(STEPS):
        x0, noise, t, text, mask = _batch(rank, SMALL_COND, s)
        if model == "nan" and s == 1 and rank == 1:
            noise[1, 2, 3, 4] = float("nan")  # only rank 1's loss is non-finite at step 1
        tr.step(x0, noise, t, text, mask)
    sd = tr.state_dict()
    torch.cuda.synchronize()
    out[f"state{rank}"] = tr.state.cpu()
    out[f"params{rank}"] = torch.cat([v.flatten() for v in sd.values()]).cpu()
    if tr.ema is not None:
        out[f"ema{rank}"] = tr.ema.cpu()
    if rank == 0:
        out["norm"] = tr.state[0].item()
    dist.destroy_process_group()


def test_two_rank_step_matches_grad_average():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _port(), out), nprocs=world, join=True)
    from tests.golden.configs import SMALL_COND
    from sdmi.trainer import DDPMTrainer
    tr = DDPMTrainer(SMALL_COND, _init_state(SMALL_COND), "cuda", lr=1e-3)
    _reference_steps(tr, world, ema_decay=0.9999)
    _compare(tr, out, world)


def test_two_rank_dit_step_matches_grad_average():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _port(), out, "dit"), nprocs=world, join=True)
    from tests.golden.configs import SMALL_DIT
    from sdmi.trainer import DDPMTrainer
    tr = DDPMTrainer(SMALL_DIT, _dit_state(), "cuda", base="dit", lr=1e-3, ema_decay=None)
    _reference_steps(tr, world, ema_decay=None)
    _compare(tr, out, world)


def test_two_rank_nonfinite_loss_on_one_rank_skips_everywhere():
    """Only rank 1's loss is non-finite at step 1: every replica skips that step WITHOUT scaler.update() (the reference
    rule, train_ddpm_cond_celebhq_multi_gpu.py:348-352, decided by the all-reduced loss flag), so both ranks end
    bit-identical, at the update of steps 0 and 2 alone, with the loss scale untouched."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _port(), out, "nan"), nprocs=world, join=True)
    from tests.golden.configs import SMALL_COND
    from sdmi.trainer import DDPMTrainer, S_SCALE, S_STEP, S_GROWTH, S_SKIP
    assert torch.equal(out["params0"], out["params1"]) and torch.equal(out["ema0"], out["ema1"])
    for r in range(world):
        st = out[f"state{r}"]
        assert st[S_SCALE].item() == 65536.0 and int(st[S_STEP].item()) == STEPS - 1
        assert int(st[S_GROWTH].item()) == STEPS - 1 and st[S_SKIP].item() == 0.0
    tr = DDPMTrainer(SMALL_COND, _init_state(SMALL_COND), "cuda", lr=1e-3)
    _reference_steps(tr, world, ema_decay=0.9999, steps=[s for s in range(STEPS) if s != 1])
    _compare(tr, out, world)


def _reference_steps(tr, world, ema_decay, steps=None):
    """One process: per step, sum the ranks' gradients by hand, then the same clip + Adam (+ EMA) kernels."""
    from tests.golden.configs import SMALL_COND
    from sdmi import _lib, kernels as K
    L = _lib.lib()
    ws = torch.empty(L.sdmi_optim_workspace() // 4, device="cuda")
    for s in (range(STEPS) if steps is None else steps):
        gsum = torch.zeros_like(tr.store.grads)
        for r in range(world):
            x0, noise, t, text, mask = _batch(r, SMALL_COND, s)
            xt = torch.empty_like(x0)
            K.add_noise(x0, noise, t, tr.sqrt_abar, tr.sqrt_1m_abar, xt)
            pred, ctx = tr.engine.forward(xt, t, text, mask)
            dpred = tr.engine.new_dpred(2, 32, 32)
            tr.engine.loss(pred, noise, dpred, tr.state[6:7], gscale_dev=tr.state[2:3])
            tr.engine.backward(ctx, dpred)
            gsum += tr.store.grads
        tr.store.grads.copy_(gsum)
        _lib.check(L.sdmi_clip_unscale(tr.store.grads.data_ptr(), tr.store.numel, 1.0, tr.state.data_ptr(),
                                       ws.data_ptr(), 2000, 0, float(world), K._stream()), "clip")
        _lib.check(L.sdmi_adam_ema(tr.store.params.data_ptr(), tr.store.grads.data_ptr(), tr.m.data_ptr(),
                                   tr.v.data_ptr(), K._p(tr.ema), tr.store.numel, tr.state.data_ptr(), 1e-3, 0.9,
                                   0.999, 1e-8, ema_decay or 0.0, 1.0 - (ema_decay or 0.0),
                                   K._stream()), "adam")
        tr.engine.refresh_weights()
    torch.cuda.synchronize()


def _compare(tr, out, world):
    assert abs(tr.state[0].item() - out["norm"]) <= 1e-4 * out["norm"]
    mine = torch.cat([v.flatten() for v in tr.state_dict().values()]).cpu()
    for r in range(world):  # every replica holds rank 0's model after the same averaged updates
        diff = (mine - out[f"params{r}"]).abs().max().item()
        assert diff <= 1e-6, (r, diff)
        if tr.ema is not None:
            assert (tr.ema.cpu() - out[f"ema{r}"]).abs().max().item() <= 1e-6, r
