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
