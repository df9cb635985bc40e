"""Model configs used by the golden fixtures and the tests (plain dicts in the reference's
model_config format, models/unet_cond_base.py:17-27)."""


def _cond(text_dim, text=True, image=True):
    types = ([] if not text else ["text"]) + ([] if not image else ["image"])
    return {
        "condition_types": types,
        "text_condition_config": {"text_embed_model": "clip", "train_text_embed_model": False,
                                  "text_embed_dim": text_dim, "cond_drop_prob": 0.1},
        "image_condition_config": {"image_condition_input_channels": 18, "image_condition_output_channels": 3,
                                   "image_condition_h": 512, "image_condition_w": 512, "cond_drop_prob": 0.1},
    }


SMALL_UNCOND = {
    "down_channels": [64, 128, 128, 256], "mid_channels": [256, 128], "down_sample": [True, True, True],
    "attn_down": [True, True, True], "time_emb_dim": 128, "norm_channels": 32, "num_heads": 8,
    "conv_out_channels": 64, "num_down_layers": 2, "num_mid_layers": 1, "num_up_layers": 2,
}
SMALL_COND = dict(SMALL_UNCOND, condition_config=_cond(64))


def full_cond_config():
    """config/celebhq_text_image_cond.py:36-118 (c_factor = 1)."""
    return {
        "down_channels": [256, 384, 512, 768], "mid_channels": [768, 512], "down_sample": [True, True, True],
        "attn_down": [True, True, True], "time_emb_dim": 512, "norm_channels": 32, "num_heads": 16,
        "conv_out_channels": 128, "num_down_layers": 2, "num_mid_layers": 2, "num_up_layers": 2,
        "condition_config": _cond(512),
    }


def full_uncond_config():
    """config/celebhq.yaml ldm_params."""
    c = full_cond_config()
    c.pop("condition_config")
    return c


# scheduler configs: (num_timesteps, beta_start, beta_end)
SCHED_COND = (1000, 0.00085, 0.012)     # config/celebhq_text_image_cond.py:31-33
SCHED_UNCOND = (1000, 0.0015, 0.0195)   # config/celebhq.yaml diffusion_params


# ---- DiT (models/transformer.py) ----
def dit12l_config():
    """Model_DiT_12L_config.py dit_model_config: hidden 288, patch 2, t-emb 192 (build_ldm_scaling(2.58)
    of the UNet's 512), 12 layers, 9 heads x 32, image-only conditioning (ldm_condition_types=['image'])."""
    return {"hidden_size": 288, "patch_size": 2, "timestep_emb_dim": 192, "num_layers": 12, "num_heads": 9,
            "head_dim": 32, "condition_config": _cond(512, text=False, image=True)}


# small DiT with text cross-attention (CustomMultiheadAttention path, Model_DiT_9L-style) and image cond
SMALL_DIT = {"hidden_size": 96, "patch_size": 2, "timestep_emb_dim": 64, "num_layers": 2, "num_heads": 3,
             "head_dim": 32, "condition_config": _cond(64, text=True, image=True)}
SMALL_DIT_UNCOND = {"hidden_size": 64, "patch_size": 2, "timestep_emb_dim": 32, "num_layers": 2, "num_heads": 2,
                    "head_dim": 32}


# ---- VQVAE (models/vqvae.py), config/celebhq.yaml autoencoder_params ----
def vqvae_celebhq_config():
    return {"z_channels": 4, "codebook_size": 8192, "down_channels": [64, 128, 256, 256], "mid_channels": [256, 256],
            "down_sample": [True, True, True], "attn_down": [False, False, False], "norm_channels": 32,
            "num_heads": 4, "num_down_layers": 2, "num_mid_layers": 2, "num_up_layers": 2}


SMALL_VQVAE = {"z_channels": 4, "codebook_size": 512, "down_channels": [32, 64, 64], "mid_channels": [64, 64],
               "down_sample": [True, True], "attn_down": [False, True], "norm_channels": 16, "num_heads": 2,
               "num_down_layers": 1, "num_mid_layers": 1, "num_up_layers": 1}


# class conditioning (unet_cond_base.py:152-155, transformer.py:176-181; tools/*class_cond*: MNIST, 10 classes)
def _class_cond(n=10):
    return {"condition_types": ["class"], "class_condition_config": {"num_classes": n, "cond_drop_prob": 0.1}}


SMALL_CLASS_UNET = dict(SMALL_UNCOND, condition_config=_class_cond())
SMALL_CLASS_DIT = dict(SMALL_DIT_UNCOND, condition_config=_class_cond())


# ---- BASELINE config 1: MNIST unconditional LDM (tools/train_ddpm_vqvae.py, default --config config/mnist.yaml).
# config/mnist.yaml is NOT in the reference tree, so these are BUILD-AUTHORED values in the
# reference's yaml schema: 28x28 single-channel images -> VQVAE (two stride-2 levels) -> 3 x 7 x 7 latents -> an
# unconditional UNet that does not down-sample (7 is odd: a stride-2 level would break the skip concatenation).
MNIST_VQVAE = {"z_channels": 3, "codebook_size": 20, "down_channels": [32, 64, 128], "mid_channels": [128, 128],
               "down_sample": [True, True], "attn_down": [False, False], "norm_channels": 32, "num_heads": 16,
               "num_down_layers": 1, "num_mid_layers": 1, "num_up_layers": 1}
MNIST_LDM = {"down_channels": [64, 128, 128], "mid_channels": [128, 128], "down_sample": [False, False],
             "attn_down": [True, True], "time_emb_dim": 128, "norm_channels": 32, "num_heads": 8,
             "conv_out_channels": 64, "num_down_layers": 1, "num_mid_layers": 1, "num_up_layers": 1}
MNIST_SCHED = (1000, 0.0015, 0.0195)
MNIST_LR = 1e-5
