"""Pins the VQVAE oracle (oracle/vqvae_oracle.py) against golden vectors produced by the reference VQVAE
itself (tests/golden/make_golden_dit_vqvae.py). CPU only.

Tolerances: quantize indices bit-exact on identical fp32 inputs (cdist + first-minimum argmin); encoder /
decoder outputs are fp32 restatements (conv blocking may differ from aten): max|diff| <= 1e-5 * max|ref|,
and the codebook indices of the full encode must match exactly."""
import os

import pytest
import torch
from safetensors.torch import load_file

from oracle import sd_oracle as O
from oracle import vqvae_oracle as VO
from tests.golden.configs import SMALL_VQVAE, vqvae_celebhq_config

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fx(name):
    return load_file(os.path.join(G, name + ".safetensors"))


def rel(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


def test_quantize_bit_exact():
    f = fx("vqvae_quantize")
    sd = O.deterministic_state(VO.vqvae_param_shapes(vqvae_celebhq_config()), seed=8)
    q, loss, idx = VO.quantize(sd, f["z"])
    assert torch.equal(idx, f["indices"])
    assert torch.equal(q, f["quant"])
    assert torch.equal(loss.reshape(1), f["codebook_loss"]) and torch.equal(loss.reshape(1), f["commitment_loss"])


@pytest.mark.parametrize("name,cfg,seed", [("vqvae_small", SMALL_VQVAE, 9), ("vqvae_celebhq", vqvae_celebhq_config(), 8)])
def test_encode_decode(name, cfg, seed):
    f = fx(name)
    sd = O.deterministic_state(VO.vqvae_param_shapes(cfg), seed=seed)
    with torch.no_grad():
        pre = VO.encode_pre_quant(sd, cfg, f["x"])
        assert rel(pre, f["pre_quant"]) <= 1e-5
        zq, losses, idx = VO.encode(sd, cfg, f["x"])
        assert torch.equal(idx, f["indices"])
        assert rel(zq, f["zq"]) <= 1e-5
        out = VO.decode(sd, cfg, zq)
        assert rel(out, f["out"]) <= 1e-5
    assert rel(losses["codebook_loss"].reshape(1), f["codebook_loss"]) <= 1e-4


def test_train_step_grads_and_adam():
    """The training restatement (quantize_train / train_grads / adam_steps) against the reference's own generator
    step (train_vqvae_celebhq.py:414-466 without LPIPS / GAN): the three loss terms, the indices, every parameter's
    gradient norm, selected full gradients, and the parameters after two Adam(2e-5, (0.5, 0.999)) steps."""
    f = fx("vqvae_train")
    sd = O.deterministic_state(VO.vqvae_param_shapes(SMALL_VQVAE), seed=9)
    seq = []
    cur = sd
    for step in range(2):
        losses, grads, out, idx = VO.train_grads(cur, SMALL_VQVAE, f[f"s{step}.im"])
        assert torch.equal(idx, f[f"s{step}.indices"])
        for k in ("recon", "codebook", "commitment"):
            assert rel(losses[k].reshape(1), f[f"s{step}.{k}"]) <= 1e-5, (step, k)
        if step == 0:
            assert rel(out, f["s0.out"]) <= 1e-5
            norms = torch.stack([grads[k].norm() for k in sd])
            assert ((norms - f["s0.grad_norms"]).abs() <= 1e-4 * f["s0.grad_norms"] + 1e-9).all()
            for k in sd:
                if "grad." + k in f:
                    g = grads[k].reshape(-1)[:8192]
                    assert rel(g, f["grad." + k]) <= 1e-4, k
        seq.append(grads)
        cur = VO.adam_steps(sd, seq)
    for k in sd:
        if "param." + k in f:
            p = cur[k].reshape(-1)[:8192]
            # Adam normalises each element's update to ~lr: gradients equal to ~1e-4 relative move an element's
            # update by a small fraction of lr (2e-5), hence an absolute bound of 5 % of one step
            assert (p - f["param." + k]).abs().max().item() <= 1e-6, k
