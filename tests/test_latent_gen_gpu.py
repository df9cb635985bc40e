"""End-to-end latent generation (reference gen_vqvae_latents.py:89-106 -> utils/diffusion_utils.py:7-18 ->
the LDM trainer): images -> models.vqvae.VQVAE.encode on the HIP path -> `.sdlat` shards of `shard_size` images
-> ResidentLatentSet in HBM -> a batch gathered on the device -> one uncond-UNet DDPM training step.

Checks: every shard record is the encoder output of its image (bit-identical to encoding the same batch
directly), the records follow the image order across numbered shards, the quantised latents agree with the fp32
oracle's encoder (same code for >= 85 % of latent pixels: random weights leave near ties; equal to 1e-5 where
the code agrees), and the gathered batch trains."""
import os

import pytest
import torch

from oracle import sd_oracle as O
from oracle import vqvae_oracle as VO
from tests.golden.configs import SMALL_UNCOND, SMALL_VQVAE

pytestmark = pytest.mark.gpu


def test_images_to_shards_to_resident_set_to_train_step(tmp_path):
    from models.vqvae import VQVAE
    from sdmi import latents as LT
    from sdmi.trainer import DDPMTrainer
    sd = O.deterministic_state(VO.vqvae_param_shapes(SMALL_VQVAE), seed=9)
    vq = VQVAE(3, SMALL_VQVAE).cuda().eval()
    vq.load_state_dict(sd)
    g = torch.Generator().manual_seed(77)
    N = 40
    ims = torch.rand(N, 3, 64, 64, generator=g) * 2 - 1
    names = [f"CelebAMask-HQ/CelebA-HQ-img/{i}.jpg" for i in range(N)]
    # host images, as a data loader yields them: generate_latents moves each batch to the encoder's device
    paths = LT.generate_latents(vq.encode, ims.cpu(), names, str(tmp_path / "lat"), shard_size=16, batch_size=8)
    assert [os.path.basename(p) for p in paths] == ["0.sdlat", "1.sdlat", "2.sdlat"]
    got = LT.load_latents(str(tmp_path / "lat"))
    assert list(got) == names
    with torch.no_grad():
        direct = torch.cat([vq.encode(ims[s:s + 8].cuda())[0].cpu() for s in range(0, N, 8)])
    for i, k in enumerate(names):
        assert torch.equal(got[k], direct[i]), k
    # against the fp32 oracle encoder + quantiser
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    with torch.no_grad():
        zq_ref, _, idx_ref = VO.encode(sd, SMALL_VQVAE, ims)
    # the codes of the same batches of 8 (a different batch size may pick other GEMM splits: other roundings)
    idx = torch.cat([vq.quantize_indices(ims[s:s + 8].cuda())[2].cpu() for s in range(0, N, 8)])
    same = (idx.cpu() == idx_ref)
    assert same.float().mean().item() >= 0.85
    m = same[:, None].expand_as(zq_ref)
    assert (direct[m] - zq_ref[m]).abs().max().item() <= 1e-5
    # HBM-resident set -> device gather -> one training step of the uncond LDM on those latents
    rs = LT.ResidentLatentSet(str(tmp_path / "lat"), names=names, device="cuda")
    sel = torch.tensor([5, 39, 0, 17], device="cuda")
    x0, _ = rs.batch(sel)
    assert torch.equal(x0.cpu(), direct[sel.cpu()])
    import models.unet_base as mu
    tr = DDPMTrainer(SMALL_UNCOND, mu.Unet(4, SMALL_UNCOND).state_dict(), "cuda", base="uncond", lr=5e-6,
                     ema_decay=None, max_grad_norm=float("inf"), sched=(1000, 0.0015, 0.0195))
    noise = torch.randn(x0.shape, generator=torch.Generator().manual_seed(1)).cuda()
    t = torch.randint(0, 1000, (4,), generator=torch.Generator().manual_seed(2)).cuda()
    tr.step(x0, noise, t)
    loss = tr.loss().item()
    assert 0.1 < loss < 10.0
