"""The drop-in nn.Module driven exactly as the reference's trainer and samplers drive theirs.

* train_ddpm_cond_celebhq_multi_gpu.py:341-378: torch.autocast(bf16) around forward + nn.MSELoss, a
  torch.amp.GradScaler (init scale 65536), scaler.scale(loss).backward(), scaler.unscale_, clip_grad_norm_(1.0),
  scaler.step(torch.optim.Adam(lr 1e-5)), scaler.update(), EMA(0.9999) over a second module's parameters -- two
  steps against the reference's own two fp32 steps (tests/golden/train_step_small_cond.safetensors): loss within
  1 %, pre-clip gradient norm within 5 %, parameter and EMA updates with cosine >= 0.9 per fixture key.
* tools/sample_ddpm_vqvae.py:29-52 style inference under torch.no_grad: the weights are packed once, not per call
  (parameter version counters unchanged), and no backward tape is kept; outputs equal the grad-enabled forward."""
import os

import pytest
import torch

from oracle import sd_oracle as O
from tests.golden.configs import SMALL_COND

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def one_hot(cmap, n=18):
    return torch.nn.functional.one_hot(cmap.long().clamp(0, n), n + 1).movedim(-1, 1)[:, 1:].float()


def cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


def _model(sd):
    import models.unet_cond_base as mc
    m = mc.Unet(4, SMALL_COND)
    m.load_state_dict(sd)
    return m.cuda()


def test_reference_trainer_loop_with_autocast_gradscaler_adam_ema():
    from safetensors.torch import load_file
    f = load_file(os.path.join(G, "train_step_small_cond.safetensors"))
    sd0 = O.deterministic_state(O.unet_param_shapes(SMALL_COND), seed=1)
    model, ema_model = _model(sd0), _model(sd0)
    model.train()
    sched = O.SchedulerTables(1000, 0.00085, 0.012)  # the scheduler's fp32 add_noise (bit-exact, test_oracle_golden)
    optimizer = torch.optim.Adam(model.parameters(), lr=1e-5)
    scaler = torch.amp.GradScaler("cuda")
    criterion = torch.nn.MSELoss()
    for s in range(2):
        im, t, noise = f[f"s{s}.x0"].cuda(), f[f"s{s}.t"].cuda(), f[f"s{s}.noise"].cuda()
        cond_input = {"text": f[f"s{s}.text"].cuda(), "image": one_hot(f[f"s{s}.classmap"]).cuda()}
        optimizer.zero_grad(set_to_none=True)
        noisy_im = sched.add_noise(im.cpu(), noise.cpu(), t.cpu()).cuda()
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
            noise_pred = model(noisy_im, t, cond_input=cond_input)
            loss = criterion(noise_pred, noise)
        assert torch.isfinite(loss)
        scaler.scale(loss).backward()
        scaler.unscale_(optimizer)
        grad_norm = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        assert torch.isfinite(grad_norm)
        scaler.step(optimizer)
        scaler.update()
        with torch.no_grad():
            for ema_param, param in zip(ema_model.parameters(), model.parameters()):
                ema_param.data.mul_(0.9999).add_(param.data, alpha=1 - 0.9999)
        rl, rn = f[f"s{s}.loss"].item(), f[f"s{s}.grad_norm"].item()
        assert abs(loss.item() - rl) <= 1e-2 * rl, (s, loss.item(), rl)
        assert abs(grad_norm.item() - rn) <= 5e-2 * rn, (s, grad_norm.item(), rn)
    assert scaler.get_scale() == 65536.0
    params, emas = dict(model.named_parameters()), dict(ema_model.named_parameters())
    for k in f:
        if not k.startswith("param."):
            continue
        key = k[6:]
        n = f[k].numel()
        init = sd0[key].reshape(-1)[:n]
        for mine, want, what in ((params[key], f[k], "param"), (emas[key], f["ema." + key], "ema")):
            d_hip = mine.detach().reshape(-1)[:n].cpu().double() - init.double()
            d_ref = want.double() - init.double()
            assert cos(d_hip, d_ref) >= 0.9, (what, key, cos(d_hip, d_ref))
            assert abs(d_hip.norm() - d_ref.norm()) <= 0.1 * d_ref.norm(), (what, key)


def test_inference_packs_once_and_keeps_no_tape():
    sd0 = O.deterministic_state(O.unet_param_shapes(SMALL_COND), seed=4)
    model = _model(sd0)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 4, 32, 32, generator=g).cuda()
    cond = {"text": torch.randn(2, 77, 64, generator=g).cuda(),
            "image": one_hot(torch.randint(0, 19, (2, 64, 64), generator=g)).cuda()}
    ref = model(x, torch.tensor([7, 300]).cuda(), cond).detach()  # grad-enabled path (packs the weights)
    eng = model._sdmi.engine
    calls = []
    orig = eng.refresh_weights
    eng.refresh_weights = lambda: (calls.append(1), orig())[1]
    with torch.no_grad():
        outs = [model(x, torch.tensor([7, 300]).cuda(), cond) for _ in range(3)]
    torch.cuda.synchronize()
    assert calls == [], "weights repacked although no parameter changed"
    for o in outs:
        assert o.grad_fn is None
        assert torch.equal(o, ref)
    with torch.no_grad():  # an in-place parameter update must trigger exactly one repack
        model.conv_out.bias.add_(0.5)
        o2 = model(x, torch.tensor([7, 300]).cuda(), cond)
        o3 = model(x, torch.tensor([7, 300]).cuda(), cond)
    torch.cuda.synchronize()
    assert len(calls) == 1
    assert torch.allclose(o2, ref + 0.5, atol=1e-5) and torch.equal(o2, o3)


def test_data_writes_between_forwards_are_seen():
    """Updates written through `.data` keep the version counter (the reference's EMA `.data.mul_().add_()`,
    PercentOptimizerFP's `p.data.copy_`): a grad-enabled forward always repacks, so its output follows the new
    weights; under torch.no_grad, sdmi_invalidate() forces the repack."""
    sd0 = O.deterministic_state(O.unet_param_shapes(SMALL_COND), seed=6)
    model = _model(sd0)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 4, 32, 32, generator=g).cuda()
    cond = {"text": torch.randn(2, 77, 64, generator=g).cuda(),
            "image": one_hot(torch.randint(0, 19, (2, 64, 64), generator=g)).cuda()}
    t = torch.tensor([5, 900]).cuda()
    a = model(x, t, cond).detach().clone()
    w = model.downs[0].resnet_conv_first[0][2].weight
    v0 = w._version
    w.data.copy_(w.data * 1.5)
    assert w._version == v0  # no version bump: the old gate would have kept the stale pack
    b = model(x, t, cond).detach()
    assert not torch.equal(a, b)
    with torch.no_grad():
        c = model(x, t, cond)
        w.data.mul_(2.0)
        stale = model(x, t, cond)
        model.sdmi_invalidate()
        d = model(x, t, cond)
    torch.cuda.synchronize()
    assert torch.equal(b, c) and torch.equal(stale, c) and not torch.equal(d, c)
    ref = model(x, t, cond).detach()  # grad-enabled: repacks, same weights as d
    assert torch.equal(ref, d)
