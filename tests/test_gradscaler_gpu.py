"""The device-side GradScaler / skip state machine of the training step (csrc/optim.hip norm_finalize_kernel +
adam_ema_kernel; reference train_ddpm_cond_celebhq_multi_gpu.py:341-378):

* non-finite loss -> the step is skipped BEFORE scaler.update() (:348-352): parameters, Adam moments, EMA, step count,
  loss scale and growth tracker all unchanged;
* finite loss, non-finite gradients -> clip_grad_norm_ returns a non-finite norm, optimizer.step and the EMA are
  skipped but scaler.update() runs (:366-371): the scale halves and the growth tracker resets;
* `growth_interval` consecutive clean steps double the scale (GradScaler defaults, :269, :374).

Checked (1) against torch.amp.GradScaler driving torch.optim.Adam + clip_grad_norm_ + the reference's EMA loop on the
same gradient sequence, and (2) through sdmi.trainer.DDPMTrainer on the model with injected NaNs."""
import pytest
import torch

from oracle import sd_oracle as O
from tests.golden.configs import SMALL_COND

pytestmark = pytest.mark.gpu


def test_state_machine_matches_torch_gradscaler_adam():
    from sdmi import _lib, kernels as K
    from sdmi.trainer import S_SCALE, S_GROWTH, S_STEP, S_SKIP, S_LOSS
    L = _lib.lib()
    n, gi = 4099, 3  # ragged length (vector body + scalar tail); growth every 3 clean steps
    g = torch.Generator().manual_seed(3)
    p0 = torch.randn(n, generator=g)
    # the sequence: clean steps, a non-finite loss, a non-finite gradient, then enough clean steps to grow twice
    events = ["ok", "ok", "nan_loss", "ok", "nan_grad", "ok", "ok", "ok", "inf_loss", "ok", "ok", "ok", "inf_grad", "ok"]
    grads = [torch.randn(n, generator=g) * (10.0 ** (i % 3 - 1)) for i in range(len(events))]
    # torch side: the reference's loop (GradScaler(init 65536, growth_interval gi), Adam(1e-3), clip 1.0, EMA 0.99)
    p_t = torch.nn.Parameter(p0.clone().cuda())
    ema_t = p0.clone().cuda()
    opt = torch.optim.Adam([p_t], lr=1e-3)
    scaler = torch.amp.GradScaler("cuda", init_scale=65536.0, growth_interval=gi)
    # HIP side
    params, m, v, ema = p0.clone().cuda(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda"), p0.clone().cuda()
    state = torch.tensor([0, 0, 65536.0, 0, 0, 0, 0, 0], dtype=torch.float32, device="cuda")
    ws = torch.empty(L.sdmi_optim_workspace() // 4, device="cuda")
    decay = 0.99
    for i, (ev, gr) in enumerate(zip(events, grads)):
        loss = float("nan") if ev == "nan_loss" else float("inf") if ev == "inf_loss" else 1.0
        bad_grad = ev in ("nan_grad", "inf_grad")
        # ---- torch ----
        t_skip = False
        if ev in ("nan_loss", "inf_loss"):
            opt.zero_grad(set_to_none=True)
            t_skip = True
        else:
            scaler.scale(torch.ones((), device="cuda"))  # the reference's scaler.scale(loss) (lazily creates the scale)
            gs = gr.cuda() * scaler.get_scale()
            if bad_grad:
                gs[17] = float("nan") if ev == "nan_grad" else float("inf")
            p_t.grad = gs
            scaler.unscale_(opt)
            norm = torch.nn.utils.clip_grad_norm_([p_t], 1.0)
            if not torch.isfinite(norm):
                opt.zero_grad(set_to_none=True)
                scaler.update()
                t_skip = True
            else:
                scaler.step(opt)
                scaler.update()
                with torch.no_grad():
                    ema_t.mul_(decay).add_(p_t.data, alpha=1 - decay)
        # ---- HIP (scaled gradients as the backward leaves them: loss x state scale) ----
        state[S_LOSS] = loss
        hg = gr.cuda() * state[S_SCALE]
        if bad_grad:
            hg[17] = float("nan") if ev == "nan_grad" else float("inf")
        _lib.check(L.sdmi_clip_unscale(hg.data_ptr(), n, 1.0, state.data_ptr(), ws.data_ptr(), gi, 1, 1.0,
                                       K._stream()), "clip")
        _lib.check(L.sdmi_adam_ema(params.data_ptr(), hg.data_ptr(), m.data_ptr(), v.data_ptr(), ema.data_ptr(), n,
                                   state.data_ptr(), 1e-3, 0.9, 0.999, 1e-8, decay, 1 - decay, K._stream()), "adam")
        torch.cuda.synchronize()
        st = state.cpu()
        assert bool(st[S_SKIP].item()) == t_skip, (i, ev)
        assert st[S_SCALE].item() == scaler.get_scale(), (i, ev, st[S_SCALE].item(), scaler.get_scale())
        assert int(st[S_GROWTH].item()) == int(scaler._growth_tracker.item()), (i, ev)
        ostep = opt.state[p_t]["step"].item() if p_t in opt.state else 0
        assert int(st[S_STEP].item()) == int(ostep), (i, ev)
        # clip coefficients come from a double-accumulated (HIP) vs fp32 (torch) norm: a few ulp apart
        assert torch.allclose(params, p_t.data, rtol=2e-6, atol=1e-7), (i, ev, (params - p_t.data).abs().max().item())
        assert torch.allclose(ema, ema_t, rtol=2e-6, atol=1e-7), (i, ev)
        if p_t in opt.state:
            assert torch.allclose(m, opt.state[p_t]["exp_avg"], rtol=1e-5, atol=1e-9), (i, ev)
            # v = g^2 doubles the clip coefficient's relative difference
            assert torch.allclose(v, opt.state[p_t]["exp_avg_sq"], rtol=4e-5, atol=1e-12), (i, ev)
    # the sequence grew the scale three times and backed it off twice: 65536 * 2 / 2 * 2 * 2 / 2
    assert scaler.get_scale() == 131072.0 and state[S_SCALE].item() == 131072.0


def _batch(seed, B=2):
    g = torch.Generator().manual_seed(seed)
    x0 = torch.randn(B, 4, 32, 32, generator=g)
    noise = torch.randn(B, 4, 32, 32, generator=g)
    t = torch.randint(0, 1000, (B,), generator=g)
    text = torch.randn(B, 77, 64, generator=g)
    cmap = torch.randint(0, 19, (B, 64, 64), generator=g)
    mask = torch.nn.functional.one_hot(cmap, 19).movedim(-1, 1)[:, 1:].float()
    return [v.cuda() for v in (x0, noise, t, text, mask)]


def test_trainer_skips_and_scales_on_injected_nans():
    """DDPMTrainer on the model: a NaN in the noise target (non-finite loss), a NaN written into the gradients after the
    backward (finite loss, non-finite norm) and growth after `growth_interval` clean steps."""
    from sdmi.trainer import DDPMTrainer, S_SCALE, S_GROWTH, S_STEP, S_SKIP, S_LOSS
    sd0 = O.deterministic_state(O.unet_param_shapes(SMALL_COND), seed=1)
    tr = DDPMTrainer(SMALL_COND, sd0, "cuda", lr=1e-3, growth_interval=3)

    def snap():
        tr.sync_optimizer()
        torch.cuda.synchronize()
        return (tr.store.params.clone(), tr.m.clone(), tr.v.clone(), tr.ema.clone(), tr.state.clone())

    def same(a, b):
        return all(torch.equal(x, y) for x, y in zip(a[:4], b[:4]))

    x0, noise, t, text, mask = _batch(1)
    tr.step(x0, noise, t, text, mask)  # clean step 1
    s1 = snap()
    assert s1[4][S_SKIP] == 0 and s1[4][S_STEP] == 1 and s1[4][S_GROWTH] == 1 and s1[4][S_SCALE] == 65536.0

    x0, noise, t, text, mask = _batch(2)
    noise[0, 0, 0, 0] = float("nan")  # non-finite loss (:348-352): skip, no scaler.update()
    tr.step(x0, noise, t, text, mask)
    s2 = snap()
    assert not torch.isfinite(s2[4][S_LOSS])
    assert s2[4][S_SKIP] == 1 and s2[4][S_STEP] == 1 and s2[4][S_GROWTH] == 1 and s2[4][S_SCALE] == 65536.0
    assert same(s1, s2), "a skipped step must leave parameters, Adam moments and the EMA untouched"

    # finite loss, non-finite gradient (:366-371): skip, scale halved, growth tracker reset
    eng = tr.engine
    orig = eng.backward

    def poisoned(ctx, dpred, **kw):
        r = orig(ctx, dpred, **kw)
        tr.store.grads[5:6].fill_(float("nan"))
        return r
    eng.backward = poisoned
    x0, noise, t, text, mask = _batch(3)
    tr.step(x0, noise, t, text, mask)
    eng.backward = orig
    s3 = snap()
    assert torch.isfinite(s3[4][S_LOSS])
    assert s3[4][S_SKIP] == 1 and s3[4][S_STEP] == 1 and s3[4][S_GROWTH] == 0 and s3[4][S_SCALE] == 32768.0
    assert same(s1, s3)

    for k in range(3):  # growth_interval clean steps: the scale doubles on the third
        x0, noise, t, text, mask = _batch(10 + k)
        tr.step(x0, noise, t, text, mask)
        s = snap()
        assert s[4][S_SKIP] == 0 and s[4][S_STEP] == 2 + k
        assert s[4][S_SCALE] == (65536.0 if k == 2 else 32768.0), (k, s[4][S_SCALE])
        assert s[4][S_GROWTH] == (0 if k == 2 else k + 1)
    assert not torch.equal(s[0], s1[0]) and not torch.equal(s[3], s1[3])
