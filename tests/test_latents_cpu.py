"""Latent / mask shard format (sdmi.latents) against the oracle's restatement of the
reference's latent cache (utils/diffusion_utils.py:7-18) and mask build (dataset/celeb_dataset.py:155-180).
All checks are bit-exact (pure data movement / integer class indices)."""
import numpy as np
import torch

from oracle import sd_oracle as O
from sdmi import latents as LT


def test_latent_shard_round_trip_and_v0_semantics(tmp_path):
    g = torch.Generator().manual_seed(0)
    single = {f"img/{i}.jpg": torch.randn(1, 4, 32, 32, generator=g) for i in range(5)}  # gen_vqvae_latents.py
    multi = {f"{i}.jpg": torch.randn(4, 32, 32, generator=g) for i in range(3)}  # the multi-GPU generator
    LT.write_latent_shard(str(tmp_path / "a.sdlat"), single)
    LT.write_latent_shard(str(tmp_path / "b.sdlat"), multi)
    got = LT.load_latents(str(tmp_path))
    assert set(got) == set(single) | set(multi)
    for k, v in single.items():
        assert torch.equal(got[k], O.latent_from_cache_value(v))  # the reference's v[0]
    for k, v in multi.items():
        assert torch.equal(got[k], v)  # normalised: v[0] would have been a (32, 32) slice
    names, arr = LT.read_latent_shard(str(tmp_path / "a.sdlat"))
    assert names == list(single) and arr.shape == (5, 4, 32, 32) and arr.dtype == np.float32


def test_empty_and_bad_shards(tmp_path):
    LT.write_latent_shard(str(tmp_path / "e.sdlat"), {})
    assert LT.load_latents(str(tmp_path)) == {}
    (tmp_path / "bad.sdlat").write_bytes(b"\0" * 128)
    try:
        LT.load_latents(str(tmp_path))
        raise AssertionError("accepted a shard without the magic")
    except ValueError:
        pass
    try:
        LT.write_latent_shard(str(tmp_path / "x.sdlat"), {"a": torch.zeros(2, 4, 8, 8)})
        raise AssertionError("accepted a (2,C,H,W) latent")
    except ValueError:
        pass


def test_class_map_equals_reference_one_hot():
    g = torch.Generator().manual_seed(1)
    for (h, w, oh, ow) in ((512, 512, 512, 512), (1024, 1024, 512, 512), (300, 300, 512, 512), (77, 50, 64, 48)):
        png = torch.randint(0, 23, (h, w), generator=g).numpy()  # values > 18 exercise the clamp
        ref = O.celeb_mask(png, oh, ow, 18)
        cm = LT.class_map_from_png_array(png, oh, ow, 18)
        assert cm.dtype == torch.uint8 and cm.shape == (oh, ow) and int(cm.max()) <= 18
        assert torch.equal(LT.one_hot_from_class_map(cm, 18), ref)
        assert torch.equal(LT.one_hot_from_class_map(cm[None], 18)[0], ref)  # batched form


def test_mask_shard_and_resident_set(tmp_path):
    g = torch.Generator().manual_seed(2)
    lat = {f"d/{i}.jpg": torch.randn(1, 4, 8, 8, generator=g) for i in range(7)}
    cms = {f"{i}.jpg": torch.randint(0, 19, (16, 16), generator=g).to(torch.uint8) for i in range(7)}
    (tmp_path / "lat").mkdir()
    (tmp_path / "msk").mkdir()
    items = list(lat.items())
    LT.write_latent_shard(str(tmp_path / "lat" / "0.sdlat"), dict(items[:4]))
    LT.write_latent_shard(str(tmp_path / "lat" / "1.sdlat"), dict(items[4:]))
    LT.write_mask_shard(str(tmp_path / "msk" / "0.sdmsk"), cms)
    names = list(reversed(list(lat)))
    rs = LT.ResidentLatentSet(str(tmp_path / "lat"), names=names, mask_dir=str(tmp_path / "msk"), device="cpu")
    assert len(rs) == 7
    idx = torch.tensor([3, 0, 6, 3])
    x, m = rs.batch(idx)
    for j, i in enumerate(idx.tolist()):
        k = names[i]
        assert torch.equal(x[j], lat[k][0])
        assert torch.equal(m[j], cms[k.split("/")[-1]])  # basename lookup (celeb_dataset.py:143-146)


def test_generate_latents_shards_in_image_order(tmp_path):
    """gen_vqvae_latents.py:89-106: one record per image, a shard every `shard_size` images ({part} numbering),
    the remainder in a last shard; the encoder is any batch callable here (the HIP VQVAE in test_latent_gen_gpu)."""
    g = torch.Generator().manual_seed(3)
    ims = torch.randn(70, 3, 16, 16, generator=g)
    names = [f"celeb/{i}.jpg" for i in range(70)]
    enc = lambda x: (torch.nn.functional.avg_pool2d(x, 4).repeat(1, 2, 1, 1)[:, :4], None)  # noqa: E731
    paths = LT.generate_latents(enc, ims, names, str(tmp_path / "lat"), shard_size=8, batch_size=6)
    assert [p.split("/")[-1] for p in paths] == [f"{i}.sdlat" for i in range(9)]
    sizes = [LT.read_latent_shard(p)[1].shape[0] for p in paths]
    assert sizes == [8] * 8 + [6]
    ref = enc(ims)[0]
    got = LT.load_latents(str(tmp_path / "lat"))
    assert list(got) == names  # part order is numeric (0, 1, ..., 8), records in image order
    for i, k in enumerate(names):
        assert torch.equal(got[k], ref[i])
    rs = LT.ResidentLatentSet(str(tmp_path / "lat"), device="cpu")
    assert rs.names == names
    x, _ = rs.batch(torch.tensor([69, 0, 33]))
    assert torch.equal(x, ref[[69, 0, 33]])
    # a list of (1, C, H, W) images (the reference data loader's batch of one) gives the same shards
    LT.generate_latents(enc, [im[None] for im in ims], names, str(tmp_path / "lat2"), shard_size=8, batch_size=5)
    got2 = LT.load_latents(str(tmp_path / "lat2"))
    assert all(torch.equal(got2[k], got[k]) for k in names)
