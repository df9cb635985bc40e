"""Generates the DiT (and VQVAE) golden fixtures in tests/golden/ by importing the REFERENCE
implementation (read-only at /root/reference) in THIS container. Only input/output tensors are
committed (safetensors); weights regenerate from oracle.sd_oracle.deterministic_state.

Run:  PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_dit_vqvae.py [dit] [vqvae] [vqvae256] [vqvae_train] [sampler] [class]

The reference DIT zero-initialises adaptive_norm_layer and proj_out (models/transformer.py:147-151,
transformer_layer.py:70-71), so a freshly built reference model outputs exactly 0; the fixtures load
the seeded non-zero state instead, after checking key order and shapes against the oracle's tables.
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
from oracle import dit_oracle as DO  # noqa: E402
from tests.golden.configs import SMALL_DIT, SMALL_DIT_UNCOND, dit12l_config  # noqa: E402
from tests.golden.make_golden import one_hot_mask  # noqa: E402

torch.set_num_threads(8)


def make_dit(cfg, seed):
    import models.transformer as ref_dit
    model = ref_dit.DIT(im_channels=4, model_config=cfg)
    shapes = DO.dit_param_shapes(cfg)
    ref_sd = model.state_dict()
    assert list(ref_sd.keys()) == list(shapes.keys()), (list(ref_sd.keys())[:12], list(shapes.keys())[:12])
    for k, v in ref_sd.items():
        assert tuple(v.shape) == tuple(shapes[k]), (k, v.shape, shapes[k])
    sd = O.deterministic_state(shapes, seed)
    model.load_state_dict(sd)
    return model, sd


def dit_inputs(B, cfg, seed, mask_hw=64):
    L = DO.dit_layout(cfg)
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, 4, 32, 32, generator=g)
    t = torch.randint(0, 1000, (B,), generator=g)
    f = {"x": x, "t": t}
    cond = {}
    if L["text"]:
        f["text"] = torch.randn(B, 77, L["ctx_dim"], generator=g)
        cond["text"] = f["text"]
    if L["image"]:
        f["classmap"] = torch.randint(0, 19, (B, mask_hw, mask_hw), generator=g).to(torch.uint8)
        cond["image"] = one_hot_mask(f["classmap"])
    return f, (cond or None)


GRAD_KEYS_DIT = ("cond_conv_in.weight", "patch_embed_layer.patch_embed.0.weight", "t_proj.0.weight",
                 "t_proj.2.bias", "transformer_layers.0.attn_block.qkv_proj.weight",
                 "transformer_layers.1.attn_block.output_proj.0.bias", "transformer_layers.0.mlp_block.0.weight",
                 "transformer_layers.1.mlp_block.2.weight", "transformer_layers.0.adaptive_norm_layer.1.weight",
                 "transformer_layers.1.adaptive_norm_layer.1.bias", "transformer_layers.0.cross_attn_block.q_proj.weight",
                 "transformer_layers.1.cross_attn_block.v_proj.bias", "transformer_layers.0.context_proj.weight",
                 "adaptive_norm_layer.1.weight", "proj_out.weight", "proj_out.bias")


def gen_dit():
    # small text+image DiT: forward, loss, gradients
    for name, cfg in (("dit_small", SMALL_DIT), ("dit_small_uncond", SMALL_DIT_UNCOND)):
        model, sd = make_dit(cfg, seed=4)
        f, cond = dit_inputs(2, cfg, seed=12)
        noise = torch.randn(f["x"].shape, generator=torch.Generator().manual_seed(13))
        f["noise"] = noise
        model.zero_grad()
        out = model(f["x"], f["t"], cond_input=cond) if cond else model(f["x"], f["t"])
        loss = torch.nn.functional.mse_loss(out, noise)
        loss.backward()
        f["out"] = out.detach()
        f["loss"] = loss.detach().reshape(1)
        f["grad_norm"] = torch.norm(torch.stack([p.grad.norm() for p in model.parameters() if p.grad is not None])
                                    ).reshape(1)
        for k, p in model.named_parameters():
            if k in GRAD_KEYS_DIT:
                f["grad." + k] = p.grad.detach().reshape(-1)[:8192].clone()
        save_file({k: v.contiguous() for k, v in f.items()}, os.path.join(HERE, f"{name}.safetensors"))

    # DiT-12L (Model_DiT_12L_config) forward at batch 2
    model, sd = make_dit(dit12l_config(), seed=6)
    f, cond = dit_inputs(2, dit12l_config(), seed=14, mask_hw=512)
    with torch.no_grad():
        f["out"] = model(f["x"], f["t"], cond_input=cond)
    save_file({k: v.contiguous() for k, v in f.items()}, os.path.join(HERE, "dit12l.safetensors"))

    # two reference DiT training steps (Model_DiT_12L_train.py:300-375: Adam lr 1e-4, clip 1.0, no EMA)
    import scheduler.linear_noise_scheduler as ref_sched
    model, sd = make_dit(SMALL_DIT, seed=4)
    sched = ref_sched.LinearNoiseScheduler(1000, 0.00085, 0.012)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    f = {}
    for step in range(2):
        inp, cond = dit_inputs(2, SMALL_DIT, seed=300 + step)
        noise = torch.randn(inp["x"].shape, generator=torch.Generator().manual_seed(400 + step))
        for k, v in inp.items():
            f[f"s{step}.{k}"] = v
        f[f"s{step}.noise"] = noise
        opt.zero_grad(set_to_none=True)
        xt = sched.add_noise(inp["x"], noise, inp["t"])
        loss = torch.nn.functional.mse_loss(model(xt, inp["t"], cond_input=cond), noise)
        loss.backward()
        gn = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        f[f"s{step}.loss"] = loss.detach().reshape(1)
        f[f"s{step}.grad_norm"] = gn.detach().reshape(1)
    for k, p in model.named_parameters():
        if k in GRAD_KEYS_DIT:
            f["param." + k] = p.detach().reshape(-1)[:8192].clone()
    save_file({k: v.contiguous() for k, v in f.items()}, os.path.join(HERE, "dit_train_step.safetensors"))

    # position embedding KAT
    from models.patch_embed import get_patch_position_embedding
    save_file({"pos_288_16x16": get_patch_position_embedding(288, (16, 16), "cpu").contiguous(),
               "pos_96_16x8": get_patch_position_embedding(96, (16, 8), "cpu").contiguous()},
              os.path.join(HERE, "dit_pos.safetensors"))


def make_vqvae(cfg, seed):
    import models.vqvae as ref_vq
    from oracle import vqvae_oracle as VO
    model = ref_vq.VQVAE(im_channels=3, model_config=cfg)
    shapes = VO.vqvae_param_shapes(cfg)
    ref_sd = model.state_dict()
    assert list(ref_sd.keys()) == list(shapes.keys()), [k for k in ref_sd if k not in shapes][:5]
    for k, v in ref_sd.items():
        assert tuple(v.shape) == tuple(shapes[k]), (k, v.shape, shapes[k])
    sd = O.deterministic_state(shapes, seed)
    model.load_state_dict(sd)
    model.eval()
    return model, sd


def gen_vqvae():
    from tests.golden.configs import SMALL_VQVAE, vqvae_celebhq_config
    # quantize KAT (models/vqvae.py:93-126): identical fp32 inputs -> indices must match exactly
    model, sd = make_vqvae(vqvae_celebhq_config(), seed=8)
    g = torch.Generator().manual_seed(21)
    z = torch.randn(2, 4, 32, 32, generator=g) * 0.5
    with torch.no_grad():
        q, losses, idx = model.quantize(z)
    save_file({"z": z, "quant": q.contiguous(), "indices": idx.contiguous(), "codebook_loss": losses["codebook_loss"].reshape(1),
               "commitment_loss": losses["commitment_loss"].reshape(1)}, os.path.join(HERE, "vqvae_quantize.safetensors"))
    # full celebhq autoencoder at 128x128 (fully convolutional; the bench runs 256x256) and a small config
    for name, cfg, seed, B, hw in (("vqvae_celebhq", vqvae_celebhq_config(), 8, 1, 128),
                                   ("vqvae_small", SMALL_VQVAE, 9, 2, 64)):
        model, sd = make_vqvae(cfg, seed)
        g = torch.Generator().manual_seed(22)
        x = torch.rand(B, 3, hw, hw, generator=g) * 2 - 1
        pre = {}
        h = model.pre_quant_conv.register_forward_hook(lambda m, i, o: pre.__setitem__("z", o.detach().clone()))
        with torch.no_grad():
            out, zq, losses = model(x)
        h.remove()
        _, _, idx = model.quantize(pre["z"])
        f = {"x": x, "pre_quant": pre["z"], "zq": zq, "indices": idx, "out": out,
             "codebook_loss": losses["codebook_loss"].reshape(1)}
        save_file({k: v.contiguous() for k, v in f.items()}, os.path.join(HERE, f"{name}.safetensors"))


def gen_vqvae256():
    """The celebhq autoencoder at its bench size (256x256, config 2), batch 1: encoder latent, indices, decoder."""
    from tests.golden.configs import vqvae_celebhq_config
    model, sd = make_vqvae(vqvae_celebhq_config(), 8)
    g = torch.Generator().manual_seed(23)
    x = torch.rand(1, 3, 256, 256, generator=g) * 2 - 1
    pre = {}
    h = model.pre_quant_conv.register_forward_hook(lambda m, i, o: pre.__setitem__("z", o.detach().clone()))
    with torch.no_grad():
        out, zq, losses = model(x)
    h.remove()
    _, _, idx = model.quantize(pre["z"])
    f = {"x": x, "pre_quant": pre["z"], "zq": zq, "indices": idx, "out": out,
         "codebook_loss": losses["codebook_loss"].reshape(1)}
    save_file({k: v.contiguous() for k, v in f.items()}, os.path.join(HERE, "vqvae_celebhq256.safetensors"))


GRAD_KEYS_VQVAE = ("encoder_conv_in.weight", "encoder_conv_in.bias", "encoder_layers.0.resnet_conv_first.0.0.weight",
                   "encoder_layers.0.down_sample_conv.weight", "encoder_layers.1.attentions.0.in_proj_weight",
                   "encoder_layers.1.attention_norms.0.weight", "encoder_mids.0.resnet_conv_second.1.2.bias",
                   "encoder_mids.0.attentions.0.out_proj.bias", "encoder_norm_out.weight", "encoder_conv_out.weight",
                   "encoder_conv_out.bias", "pre_quant_conv.weight", "pre_quant_conv.bias", "embedding.weight",
                   "post_quant_conv.weight", "post_quant_conv.bias", "decoder_conv_in.weight", "decoder_conv_in.bias",
                   "decoder_mids.0.resnet_conv_first.0.2.weight", "decoder_layers.0.up_sample_conv.weight",
                   "decoder_layers.0.up_sample_conv.bias", "decoder_layers.0.attentions.0.out_proj.weight",
                   "decoder_layers.1.residual_input_conv.0.weight", "decoder_norm_out.weight",
                   "decoder_conv_out.weight", "decoder_conv_out.bias")


def gen_vqvae_train():
    """Generator step of train_vqvae_celebhq.py:414-466 on the small config (no LPIPS / GAN): loss terms, every
    parameter's gradient norm, selected gradients, and the parameters after two Adam(2e-5, (0.5, 0.999)) steps."""
    from tests.golden.configs import SMALL_VQVAE
    model, sd = make_vqvae(SMALL_VQVAE, 9)
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=2e-5, betas=(0.5, 0.999))
    f = {}
    for step in range(2):
        g = torch.Generator().manual_seed(60 + step)
        im = torch.rand(2, 3, 64, 64, generator=g) * 2 - 1
        pre = {}
        h = model.pre_quant_conv.register_forward_hook(lambda m, i, o: pre.__setitem__("z", o.detach().clone()))
        opt.zero_grad()
        out, _, ql = model(im)
        h.remove()
        recon = torch.nn.functional.mse_loss(out, im)
        cb, cm = 1.0 * ql["codebook_loss"], 0.2 * ql["commitment_loss"]
        total = recon + cb + cm
        total.backward()
        with torch.no_grad():
            _, _, idx = model.quantize(pre["z"])
        f.update({f"s{step}.im": im, f"s{step}.recon": recon.detach().reshape(1), f"s{step}.codebook": cb.detach().reshape(1),
                  f"s{step}.commitment": cm.detach().reshape(1), f"s{step}.indices": idx, f"s{step}.pre_quant": pre["z"]})
        if step == 0:
            f["s0.out"] = out.detach()
            f["s0.grad_norms"] = torch.stack([p.grad.norm() if p.grad is not None else torch.zeros(())
                                              for _, p in model.named_parameters()])
            for k, p in model.named_parameters():
                if k in GRAD_KEYS_VQVAE:
                    f["grad." + k] = p.grad.detach().reshape(-1)[:8192].clone()
        opt.step()
    for k, p in model.named_parameters():
        if k in GRAD_KEYS_VQVAE:
            f["param." + k] = p.detach().reshape(-1)[:8192].clone()
    save_file({k: v.contiguous() for k, v in f.items()}, os.path.join(HERE, "vqvae_train.safetensors"))


def gen_sampler():
    """DDIMSampler / DDPMSampler steps (scheduler/linear_noise_scheduler.py:93-232) with a fixed-output model
    and fixed noise (torch.randn_like patched), so the step arithmetic alone is pinned."""
    import scheduler.linear_noise_scheduler as S
    g = torch.Generator().manual_seed(31)
    x = torch.randn(2, 4, 8, 8, generator=g)
    eps = torch.randn(2, 4, 8, 8, generator=g)
    noise = torch.randn(2, 4, 8, 8, generator=g)
    f = {"x": x, "eps": eps, "noise": noise}

    class Fixed(torch.nn.Module):
        def forward(self, *a, **k):
            return eps.clone()

    real = torch.randn_like
    torch.randn_like = lambda t, *a, **k: noise.clone()
    try:
        ddim = S.DDIMSampler(Fixed(), beta=(0.00085, 0.012), T=1000)
        ddim.cond_input = None
        for eta in (0.0, 1.0):
            for (t, tp) in ((801, 760), (11, 1), (1, 0)):
                f[f"ddim_eta{eta:g}_{t}_{tp}"] = ddim.sample_one_step(x, t, tp, eta)
        f["ddim_alpha_t_bar"] = ddim.alpha_t_bar.clone()
        ddpm = S.DDPMSampler(Fixed(), beta=(0.0001, 0.02), T=1000)
        for k in ("coeff_1", "coeff_2", "posterior_variance"):
            f[f"ddpm_{k}"] = getattr(ddpm, k).clone()  # host-CPU cumprod rounding varies by CPU: pin the tables
        for t in (999, 500, 0):
            f[f"ddpm_{t}"] = ddpm.sample_one_step(x, t)
    finally:
        torch.randn_like = real
    save_file({k: v.contiguous() for k, v in f.items()}, os.path.join(HERE, "samplers.safetensors"))


def gen_class():
    """Class-conditional small UNet and DiT (10 classes, soft + one-hot rows): forward, loss, gradients incl.
    class_emb.weight."""
    import models.unet_cond_base as ref_cond
    from tests.golden.configs import SMALL_CLASS_UNET, SMALL_CLASS_DIT
    from tests.golden.make_golden import make_model
    g = torch.Generator().manual_seed(41)
    x = torch.randn(2, 4, 32, 32, generator=g)
    t = torch.randint(0, 1000, (2,), generator=g)
    klass = torch.zeros(2, 10)
    klass[0, 3] = 1.0
    klass[1] = torch.rand(10, generator=g)  # soft row: the einsum takes any weights
    noise = torch.randn(2, 4, 32, 32, generator=g)
    for name, build in (("unet_class_small", lambda: make_model(ref_cond, SMALL_CLASS_UNET, seed=5)),
                        ("dit_class_small", lambda: make_dit(SMALL_CLASS_DIT, seed=6))):
        model, sd = build()
        model.train()
        model.zero_grad()
        out = model(x, t, cond_input={"class": klass})
        loss = torch.nn.functional.mse_loss(out, noise)
        loss.backward()
        f = {"x": x, "t": t, "class": klass, "noise": noise, "out": out.detach(), "loss": loss.detach().reshape(1)}
        for k, p in model.named_parameters():
            if k in ("class_emb.weight", "t_proj.0.weight", "t_proj.2.bias"):
                f["grad." + k] = p.grad.detach().clone()
        save_file({k: v.contiguous() for k, v in f.items()}, os.path.join(HERE, f"{name}.safetensors"))


def main():
    what = sys.argv[1:] or ["dit", "vqvae", "sampler", "class"]
    if "dit" in what:
        gen_dit()
    if "vqvae" in what:
        gen_vqvae()
    if "vqvae256" in what:
        gen_vqvae256()
    if "vqvae_train" in what:
        gen_vqvae_train()
    if "sampler" in what:
        gen_sampler()
    if "class" in what:
        gen_class()
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
