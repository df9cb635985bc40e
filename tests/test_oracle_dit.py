"""Pins the DiT oracle (oracle/dit_oracle.py) against golden vectors produced by the reference DIT itself
(tests/golden/make_golden_dit_vqvae.py). CPU only.

Tolerances: position embedding bit-exact (same fp32 op order); model outputs / gradients / optimizer
steps are fp32 restatements whose matmul blocking may differ from aten's: max|diff| <= 1e-5 * max|ref|
(2e-5 for gradients accumulated through 12 layers / two Adam steps)."""
import os

import pytest
import torch
from safetensors.torch import load_file

from oracle import sd_oracle as O
from oracle import dit_oracle as DO
from tests.golden.configs import SMALL_DIT, SMALL_DIT_UNCOND, SCHED_COND, dit12l_config

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fx(name):
    return load_file(os.path.join(G, name + ".safetensors"))


def one_hot(cmap, n=18):
    return torch.nn.functional.one_hot(cmap.long().clamp(0, n), n + 1).movedim(-1, 1)[:, 1:].float()


def rel(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


def cond_of(f):
    c = {}
    if "text" in f:
        c["text"] = f["text"]
    if "classmap" in f:
        c["image"] = one_hot(f["classmap"])
    return c or None


def test_position_embedding_bit_exact():
    f = fx("dit_pos")
    assert torch.equal(DO.patch_position_embedding(288, 16, 16), f["pos_288_16x16"])
    assert torch.equal(DO.patch_position_embedding(96, 16, 8), f["pos_96_16x8"])


def test_patchify_roundtrip():
    x = torch.randn(2, 7, 8, 6)
    t = DO.patchify(x, 2)
    assert t.shape == (2, 12, 28)
    assert torch.equal(t[0, 0, :7], x[0, :, 0, 0]) and torch.equal(t[0, 0, 7:14], x[0, :, 0, 1])
    assert torch.equal(DO.unpatchify(t, 7, 8, 6, 2), x)


@pytest.mark.parametrize("name,cfg", [("dit_small", SMALL_DIT), ("dit_small_uncond", SMALL_DIT_UNCOND)])
def test_small_dit_forward_and_grads(name, cfg):
    f = fx(name)
    sd = O.deterministic_state(DO.dit_param_shapes(cfg), seed=4)
    leaves = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    out = DO.dit_forward(leaves, cfg, f["x"], f["t"], cond_of(f))
    assert rel(out.detach(), f["out"]) <= 1e-5
    loss = torch.nn.functional.mse_loss(out, f["noise"])
    assert rel(loss.detach().reshape(1), f["loss"]) <= 1e-5
    loss.backward()
    norm = torch.norm(torch.stack([v.grad.norm() for v in leaves.values() if v.grad is not None]))
    assert rel(norm.reshape(1), f["grad_norm"]) <= 1e-5
    n = 0
    for k in f:
        if k.startswith("grad."):
            key = k[5:]
            assert rel(leaves[key].grad.reshape(-1)[:8192], f[k]) <= 2e-5, key
            n += 1
    assert n >= 8


def test_dit12l_forward():
    f = fx("dit12l")
    cfg = dit12l_config()
    sd = O.deterministic_state(DO.dit_param_shapes(cfg), seed=6)
    with torch.no_grad():
        out = DO.dit_forward(sd, cfg, f["x"], f["t"], cond_of(f))
    assert rel(out, f["out"]) <= 1e-5


def test_dit_train_step_matches_reference():
    f = fx("dit_train_step")
    sd = O.deterministic_state(DO.dit_param_shapes(SMALL_DIT), seed=4)
    opt = O.AdamState(sd)
    sched = O.SchedulerTables(*SCHED_COND)
    for s in range(2):
        inp = {k.split(".", 1)[1]: v for k, v in f.items() if k.startswith(f"s{s}.")}
        loss, norm, stepped = DO.dit_train_step(sd, opt, SMALL_DIT, sched, inp["x"], inp["noise"], inp["t"],
                                                cond_of(inp))
        assert stepped
        assert rel(loss.reshape(1), inp["loss"]) <= 1e-5
        assert rel(norm.reshape(1), inp["grad_norm"]) <= 1e-5
    for k in f:
        if k.startswith("param."):
            assert rel(sd[k[6:]].reshape(-1)[:8192], f[k]) <= 2e-5, k
