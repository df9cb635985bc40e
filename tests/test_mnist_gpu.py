"""BASELINE config 1: the MNIST unconditional LDM of tools/train_ddpm_vqvae.py:85-113 at batch 4 on the HIP path --
VQVAE encode of 1 x 28 x 28 images to 3 x 7 x 7 latents (odd spatial sizes: magic-number pixel decomposition,
3 latent channels padded to 8), then the uncond UNet step -- against the reference's own run
(tests/golden/mnist_ldm.safetensors, build-authored configs: config/mnist.yaml is absent from the reference).

Tolerances: encoder latent relative RMS <= 2e-2 and >= 90 % codebook-index agreement (20 codes); UNet forward MSE
<= 1e-4, loss within 1 %, gradient cosine >= 0.99 per fixture key, global norm within 5 %; two trainer steps
(Adam lr 1e-5, no clip, no EMA): loss 1 %, norm 5 %, parameter-update cosine >= 0.9 per fixture key."""
import os

import pytest
import torch
from safetensors.torch import load_file

from oracle import sd_oracle as O
from oracle import vqvae_oracle as VO
from tests.golden.configs import MNIST_VQVAE, MNIST_LDM, MNIST_SCHED, MNIST_LR

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


def rrms(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).pow(2).mean().sqrt() / b.pow(2).mean().sqrt()).item()


def _vae():
    from models.vqvae import VQVAE
    m = VQVAE(1, MNIST_VQVAE)
    m.load_state_dict(O.deterministic_state(VO.vqvae_param_shapes(MNIST_VQVAE, im_channels=1), seed=51))
    return m.cuda()


def _unet_state():
    return O.deterministic_state(O.unet_param_shapes(MNIST_LDM, im_channels=3, base="uncond"), seed=52)


def test_mnist_vqvae_encode():
    """Encoder to the pre-quantisation latent vs the oracle (pinned bit-exact to the reference's indices on the CPU),
    then the codebook search: indices agree with the reference's on >= 90 % of the 196 positions (bf16 moves a few
    latents across a Voronoi boundary of the 20-code book) and z_q is exactly the selected codebook rows."""
    f = load_file(os.path.join(G, "mnist_ldm.safetensors"))
    vae = _vae()
    vsd = O.deterministic_state(VO.vqvae_param_shapes(MNIST_VQVAE, im_channels=1), seed=51)
    with torch.no_grad():
        pre_ref = VO.encode_pre_quant(vsd, MNIST_VQVAE, f["s0.im"])
        z, losses = vae.encode(f["s0.im"].cuda())
        zq, _, idx, pre = vae._eng(f["s0.im"].cuda()).encode(f["s0.im"].cuda(), want_pre_quant=True)
    torch.cuda.synchronize()
    assert z.shape == (4, 3, 7, 7)
    e = rrms(pre, pre_ref)
    assert e <= 2e-2, e
    agree = (idx.cpu() == f["s0.indices"]).float().mean().item()
    assert agree >= 0.9, agree
    emb = vsd["embedding.weight"]
    assert rrms(zq, emb[idx.cpu()].permute(0, 3, 1, 2)) <= 1e-6


def test_mnist_unet_forward_backward():
    import models.unet_base as mu
    f = load_file(os.path.join(G, "mnist_ldm.safetensors"))
    model = mu.Unet(3, MNIST_LDM)
    model.load_state_dict(_unet_state())
    model = model.cuda()
    sched = O.SchedulerTables(*MNIST_SCHED)
    noisy = sched.add_noise(f["s0.z"], f["s0.noise"], f["s0.t"])
    out = model(noisy.cuda(), f["s0.t"].cuda())
    loss = torch.nn.functional.mse_loss(out, f["s0.noise"].cuda())
    loss.backward()
    torch.cuda.synchronize()
    assert ((out.detach().cpu() - f["s0.pred"]) ** 2).mean().item() <= 1e-4
    assert abs(loss.item() - f["s0.loss"].item()) <= 1e-2 * f["s0.loss"].item()
    p = dict(model.named_parameters())
    for k in f:
        if k.startswith("grad."):
            n = f[k].numel()
            c = cos(p[k[5:]].grad.reshape(-1)[:n].cpu(), f[k])
            assert c >= 0.99, (k, c)
    gn = torch.norm(torch.stack([q.grad.norm() for q in model.parameters()])).item()
    assert abs(gn - f["s0.grad_norm"].item()) <= 0.05 * f["s0.grad_norm"].item()


def test_mnist_trainer_two_steps():
    from sdmi.trainer import DDPMTrainer, S_LOSS, S_NORM
    f = load_file(os.path.join(G, "mnist_ldm.safetensors"))
    sd0 = _unet_state()
    tr = DDPMTrainer(MNIST_LDM, sd0, "cuda", base="uncond", lr=MNIST_LR, ema_decay=None,
                     max_grad_norm=float("inf"), sched=MNIST_SCHED)
    for s in range(2):
        tr.step(f[f"s{s}.z"].cuda(), f[f"s{s}.noise"].cuda(), f[f"s{s}.t"].cuda())
        torch.cuda.synchronize()
        loss, norm = tr.state[S_LOSS].item(), tr.state[S_NORM].item()
        assert abs(loss - f[f"s{s}.loss"].item()) <= 1e-2 * f[f"s{s}.loss"].item(), (s, loss)
        assert abs(norm - f[f"s{s}.grad_norm"].item()) <= 5e-2 * f[f"s{s}.grad_norm"].item(), (s, norm)
    sd = tr.state_dict()
    for k in f:
        if k.startswith("param."):
            key = k[6:]
            n = f[k].numel()
            init = sd0[key].reshape(-1)[:n]
            c = cos(sd[key].reshape(-1)[:n].cpu() - init, f[k] - init)
            assert c >= 0.9, (key, c)
