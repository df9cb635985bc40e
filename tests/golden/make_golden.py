"""Generates the golden fixtures in tests/golden/ by importing the REFERENCE implementation
(read-only at /root/reference) in THIS container. The reference never travels: only the
input/output tensors it produced are committed (safetensors), together with this script.

Run:  PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Weights come from oracle.sd_oracle.deterministic_state (seeded per state-dict key), so the fixtures
store inputs and outputs only. Every reference model's state dict is checked key-for-key and
shape-for-shape against oracle.sd_oracle.unet_param_shapes before use.
"""
import os
import sys

import torch
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
REF = os.environ.get("SDMI_REFERENCE", "/root/reference")
if REF not in sys.path:
    sys.path.insert(1, REF)

from oracle import sd_oracle as O  # noqa: E402
from tests.golden.configs import SMALL_COND, SMALL_UNCOND, full_cond_config, full_uncond_config  # noqa: E402

import models.unet_cond_base as ref_cond  # noqa: E402  (reference)
import models.unet_base as ref_uncond  # noqa: E402
import models.blocks as ref_blocks  # noqa: E402
import scheduler.linear_noise_scheduler as ref_sched  # noqa: E402

torch.set_num_threads(8)


def make_model(mod, cfg, seed):
    model = mod.Unet(im_channels=4, model_config=cfg)
    shapes = O.unet_param_shapes(cfg, base="uncond" if mod is ref_uncond else "cond")
    ref_sd = model.state_dict()
    assert list(ref_sd.keys()) == list(shapes.keys()), "state-dict key order differs from oracle layout"
    for k, v in ref_sd.items():
        assert tuple(v.shape) == tuple(shapes[k]), (k, v.shape, shapes[k])
    sd = O.deterministic_state(shapes, seed)
    model.load_state_dict(sd)
    model.eval()
    return model, sd


def one_hot_mask(classmap, n=18):
    # reference dataset builds an 18-channel one-hot mask from the class map (celeb_dataset.py:164-180)
    B, H, W = classmap.shape
    m = torch.zeros(B, n, H, W)
    for c in range(n):
        m[:, c] = (classmap == c + 1).float()  # class 0 = background -> all-zero
    return m


def inputs(B, H, ctx_dim, mask_hw, seed, T=1000):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, 4, H, H, generator=g)
    t = torch.randint(0, T, (B,), generator=g)
    text = torch.randn(B, 77, ctx_dim, generator=g) if ctx_dim else None
    cmap = torch.randint(0, 19, (B, mask_hw, mask_hw), generator=g).to(torch.uint8) if mask_hw else None
    return x, t, text, cmap


def main():
    out = {}
    # ---- scheduler tables and add_noise (bit-exact) ----
    for name, (b0, b1) in {"cond": (0.00085, 0.012), "uncond": (0.0015, 0.0195)}.items():
        s = ref_sched.LinearNoiseScheduler(1000, b0, b1)
        g = torch.Generator().manual_seed(7)
        x0 = torch.randn(8, 4, 8, 8, generator=g)
        eps = torch.randn(8, 4, 8, 8, generator=g)
        t = torch.tensor([0, 1, 17, 250, 499, 500, 998, 999])
        f = {"betas": s.betas, "alphas": s.alphas, "alpha_cum_prod": s.alpha_cum_prod,
             "sqrt_alpha_cum_prod": s.sqrt_alpha_cum_prod,
             "sqrt_one_minus_alpha_cum_prod": s.sqrt_one_minus_alpha_cum_prod,
             "x0": x0, "eps": eps, "t": t, "xt": s.add_noise(x0, eps, t)}
        # reverse step with a fixed z (monkeypatch the CPU randn used at scheduler :72)
        z = torch.randn(8, 4, 8, 8, generator=g)
        real = torch.randn
        torch.randn = lambda *a, **k: z.clone()
        try:
            xprev, x0hat = s.sample_prev_timestep(f["xt"], eps * 0.9, torch.tensor(500))
            xprev0, x0hat0 = s.sample_prev_timestep(f["xt"], eps * 0.9, torch.tensor(0))
        finally:
            torch.randn = real
        f.update(z=z, prev_500=xprev, x0hat_500=x0hat, prev_0=xprev0, x0hat_0=x0hat0)
        save_file({k: v.contiguous() for k, v in f.items()}, os.path.join(HERE, f"scheduler_{name}.safetensors"))

    # ---- time embedding ----
    t = torch.tensor([0, 1, 2, 10, 99, 500, 998, 999])
    save_file({"t": t, "emb512": ref_blocks.get_time_embedding(t, 512), "emb128": ref_blocks.get_time_embedding(t, 128)},
              os.path.join(HERE, "time_embedding.safetensors"))

    # ---- multi-head attention KAT (torch nn.MultiheadAttention as the reference uses it) ----
    f = {}
    for tag, (E, H, N, S) in {"self_d8": (128, 16, 64, 64), "self_d24": (384, 16, 16, 16),
                              "cross_d32": (512, 16, 16, 77)}.items():
        mha = torch.nn.MultiheadAttention(E, H, batch_first=True)
        mha.load_state_dict(O.deterministic_state(O.mha_param_shapes(E), seed=E + H))
        g = torch.Generator().manual_seed(11)
        q = torch.randn(2, N, E, generator=g)
        kv = q if S == N and tag.startswith("self") else torch.randn(2, S, E, generator=g)
        o, _ = mha(q, kv, kv)
        f[f"{tag}.q"] = q
        f[f"{tag}.kv"] = kv.clone()
        f[f"{tag}.out"] = o.detach()
    save_file({k: v.contiguous() for k, v in f.items()}, os.path.join(HERE, "mha.safetensors"))

    # ---- small cond / uncond UNet forward + grads ----
    for name, mod, cfg, ctx in (("small_cond", ref_cond, SMALL_COND, 64), ("small_uncond", ref_uncond, SMALL_UNCOND, 0)):
        model, sd = make_model(mod, cfg, seed=1)
        x, t, text, cmap = inputs(2, 32, ctx, 64 if ctx else 0, seed=3)
        f = {"x": x, "t": t}
        if ctx:
            f["text"] = text
            f["classmap"] = cmap
            cond = {"text": text, "image": one_hot_mask(cmap)}
            pred = model(x, t, cond_input=cond)
        else:
            pred = model(x, t)
        f["out"] = pred.detach()
        # loss + gradients of selected parameters
        model.train()
        model.zero_grad()
        noise = torch.randn(x.shape, generator=torch.Generator().manual_seed(5))
        f["noise"] = noise
        pred = model(x, t, cond_input=cond) if ctx else model(x, t)
        loss = torch.nn.functional.mse_loss(pred, noise)
        loss.backward()
        f["loss"] = loss.detach().reshape(1)
        norm = torch.norm(torch.stack([torch.norm(p.grad) for p in model.parameters() if p.grad is not None]))
        f["grad_norm"] = norm.reshape(1)
        for k, p in model.named_parameters():
            if k in GRAD_KEYS.get(name, ()):
                f["grad." + k] = p.grad.detach().reshape(-1)[:8192].clone()
        save_file({k: v.contiguous() for k, v in f.items()}, os.path.join(HERE, f"{name}.safetensors"))

    # ---- two reference training steps on the small cond model (fp32, Adam, clip, EMA) ----
    model, sd = make_model(ref_cond, SMALL_COND, seed=1)
    ema = {k: v.clone() for k, v in sd.items()}
    sched = ref_sched.LinearNoiseScheduler(1000, 0.00085, 0.012)
    opt = torch.optim.Adam(model.parameters(), lr=1e-5)
    f = {}
    model.train()
    for step in range(2):
        x, t, text, cmap = inputs(2, 32, 64, 64, seed=100 + step)
        noise = torch.randn(x.shape, generator=torch.Generator().manual_seed(200 + step))
        cond = {"text": text, "image": one_hot_mask(cmap)}
        f.update({f"s{step}.x0": x, f"s{step}.t": t, f"s{step}.text": text, f"s{step}.classmap": cmap,
                  f"s{step}.noise": noise})
        opt.zero_grad(set_to_none=True)
        xt = sched.add_noise(x, noise, t)
        loss = torch.nn.functional.mse_loss(model(xt, t, cond_input=cond), noise)
        loss.backward()
        gn = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        with torch.no_grad():
            for k, p in model.named_parameters():
                ema[k].mul_(0.9999).add_(p.data, alpha=1 - 0.9999)
        f[f"s{step}.loss"] = loss.detach().reshape(1)
        f[f"s{step}.grad_norm"] = gn.detach().reshape(1)
    for k, p in model.named_parameters():
        if k in STEP_KEYS:
            f["param." + k] = p.detach().reshape(-1)[:8192].clone()
            f["ema." + k] = ema[k].reshape(-1)[:8192].clone()
    save_file({k: v.contiguous() for k, v in f.items()}, os.path.join(HERE, "train_step_small_cond.safetensors"))

    # ---- full-size models, batch 1 (outputs only) ----
    for name, mod, cfg, ctx in (("full_cond", ref_cond, full_cond_config(), 512),
                                ("full_uncond", ref_uncond, full_uncond_config(), 0)):
        model, sd = make_model(mod, cfg, seed=2)
        x, t, text, cmap = inputs(1, 32, ctx, 512 if ctx else 0, seed=9)
        f = {"x": x, "t": t}
        with torch.no_grad():
            if ctx:
                f["text"] = text
                f["classmap"] = cmap
                pred = model(x, t, cond_input={"text": text, "image": one_hot_mask(cmap)})
            else:
                pred = model(x, t)
        f["out"] = pred
        save_file({k: v.contiguous() for k, v in f.items()}, os.path.join(HERE, f"{name}.safetensors"))
        del model, sd
    print("golden fixtures written to", HERE)


def gen_mnist():
    """BASELINE config 1 (tools/train_ddpm_vqvae.py:85-113 without cached latents): per step, images (B=4, 1 x 28 x 28 in
    [-1, 1] as MnistDataset yields them) -> vae.encode under no_grad -> add_noise -> uncond Unet -> MSE -> backward ->
    Adam(ldm_lr), no clip, no EMA. Two steps; the first also stores the loss gradients of selected parameters."""
    import models.vqvae as ref_vq
    from oracle import vqvae_oracle as VO
    from tests.golden.configs import MNIST_VQVAE, MNIST_LDM, MNIST_SCHED, MNIST_LR
    vae = ref_vq.VQVAE(im_channels=1, model_config=MNIST_VQVAE)
    shapes = VO.vqvae_param_shapes(MNIST_VQVAE, im_channels=1)
    assert list(vae.state_dict().keys()) == list(shapes.keys())
    vae.load_state_dict(O.deterministic_state(shapes, seed=51))
    vae.eval()
    model = ref_uncond.Unet(im_channels=MNIST_VQVAE["z_channels"], model_config=MNIST_LDM)
    ushapes = O.unet_param_shapes(MNIST_LDM, im_channels=3, base="uncond")
    assert list(model.state_dict().keys()) == list(ushapes.keys())
    for k, v in model.state_dict().items():
        assert tuple(v.shape) == tuple(ushapes[k]), k
    model.load_state_dict(O.deterministic_state(ushapes, seed=52))
    model.train()
    sched = ref_sched.LinearNoiseScheduler(*MNIST_SCHED)
    opt = torch.optim.Adam(model.parameters(), lr=MNIST_LR)
    f = {}
    g = torch.Generator().manual_seed(53)
    for step in range(2):
        im = torch.rand(4, 1, 28, 28, generator=g) * 2 - 1
        opt.zero_grad()
        with torch.no_grad():
            z, _ = vae.encode(im)
            _, _, idx = vae.quantize(vae.pre_quant_conv(vae.encoder_conv_out(torch.nn.SiLU()(vae.encoder_norm_out(
                _enc_trunk(vae, im))))))
        noise = torch.randn(z.shape, generator=g)
        t = torch.randint(0, MNIST_SCHED[0], (4,), generator=g)
        noisy = sched.add_noise(z, noise, t)
        pred = model(noisy, t)
        loss = torch.nn.functional.mse_loss(pred, noise)
        loss.backward()
        f.update({f"s{step}.im": im, f"s{step}.z": z, f"s{step}.indices": idx, f"s{step}.noise": noise,
                  f"s{step}.t": t, f"s{step}.pred": pred.detach(), f"s{step}.loss": loss.detach().reshape(1),
                  f"s{step}.grad_norm": torch.norm(torch.stack([p.grad.norm() for p in model.parameters()])).reshape(1)})
        if step == 0:
            for k, p in model.named_parameters():
                if k in MNIST_GRAD_KEYS:
                    f["grad." + k] = p.grad.detach().reshape(-1)[:8192].clone()
        opt.step()
    for k, p in model.named_parameters():
        if k in MNIST_GRAD_KEYS:
            f["param." + k] = p.detach().reshape(-1)[:8192].clone()
    save_file({k: v.contiguous() for k, v in f.items()}, os.path.join(HERE, "mnist_ldm.safetensors"))


def _enc_trunk(vae, x):
    out = vae.encoder_conv_in(x)
    for down in vae.encoder_layers:
        out = down(out)
    for mid in vae.encoder_mids:
        out = mid(out)
    return out


MNIST_GRAD_KEYS = ("conv_in.weight", "t_proj.0.weight", "downs.0.resnet_conv_first.0.2.weight",
                   "downs.1.attentions.0.in_proj_weight", "mids.0.resnet_conv_second.1.2.weight",
                   "ups.0.residual_input_conv.0.weight", "ups.1.attentions.0.out_proj.weight", "norm_out.weight",
                   "conv_out.weight", "conv_out.bias")


GRAD_KEYS = {
    "small_cond": ("cond_conv_in.weight", "conv_in_concat.weight", "t_proj.0.weight",
                   "downs.0.attentions.0.in_proj_weight", "downs.1.cross_attentions.0.out_proj.weight",
                   "downs.0.context_proj.0.weight", "mids.0.resnet_conv_first.0.0.weight",
                   "ups.0.up_sample_conv.weight", "ups.2.residual_input_conv.1.weight", "conv_out.weight",
                   "norm_out.weight", "downs.2.down_sample_conv.weight"),
    "small_uncond": ("conv_in.weight", "downs.0.resnet_conv_second.1.2.weight", "conv_out.bias",
                     "ups.1.attentions.1.in_proj_bias"),
}
STEP_KEYS = ("conv_in_concat.weight", "downs.0.resnet_conv_first.0.2.weight", "downs.1.attentions.0.in_proj_weight",
             "mids.0.cross_attentions.0.out_proj.bias", "ups.2.t_emb_layers.1.1.weight", "conv_out.weight",
             "norm_out.bias", "cond_conv_in.weight")

if __name__ == "__main__":
    if sys.argv[1:] == ["mnist"]:
        gen_mnist()
    else:
        main()
