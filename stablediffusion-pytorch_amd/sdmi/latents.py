"""Latent / mask shard format and an HBM-resident training set.

The reference caches VQVAE latents as pickle shards `{image_path: tensor(1, 4, 32, 32)}` of 1000 images
(gen_vqvae_latents.py:89-106) and reads them back with `load_latents` (utils/diffusion_utils.py:7-18,
keeping `v[0]`); the multi-GPU generator stores `(4, 32, 32)` per image (gen_vqvae_latents_multi_GPU.py:161),
so `v[0]` silently yields a `(32, 32)` slice there. Masks are decoded per sample from CelebAMask-HQ class PNGs
into an 18-channel fp32 one-hot at 512x512 (dataset/celeb_dataset.py:155-180: nearest resize, clamp(0, 18),
one_hot(19), background dropped) -- 18.9 MB per image.

This module replaces both with flat binary shards that load without unpickling:

* latent shard (`*.sdlat`): 64-byte header + JSON name table + one contiguous little-endian fp32 array
  `(N, C, H, W)`. Every latent is normalised to `(C, H, W)` when written (a leading singleton dim -- the
  single-GPU generator's `(1, C, H, W)` -- is dropped; `(C, H, W)` is kept as is), so both generators'
  outputs give the same shard and `load_latents` returns what the reference's `v[0]` meant.
* mask shard (`*.sdmsk`): same header + names + a uint8 class map `(N, MH, MW)` (values already clamped to
  [0, mask_channels]): 262 KB per image instead of 18.9 MB. The HIP input staging consumes class maps
  directly (`sdmi_prep_input_cmap` / `sdmi_cond_wgrad_cmap`, bit-identical to the one-hot path).
* `generate_latents`: the reference's latent generation (gen_vqvae_latents.py:89-106) batched through the HIP
  VQVAE encoder, written as `.sdlat` shards of 1000 images.
* `ResidentLatentSet`: the whole training set (latents + class maps) copied to HBM once (30k CelebHQ images =
  0.5 GB latents + 7.9 GB class maps, a few % of 288 GB); a batch is a device-side gather of row indices, no
  per-step host work or H2D copies.
"""
import glob
import json
import os
import struct

import numpy as np
import torch

MAGIC_LAT = b"SDMILAT1"
MAGIC_MSK = b"SDMIMSK1"
_HDR = struct.Struct("<8sQQIIIIQ16x")  # magic, count, names_bytes, d0, d1, d2, dtype code, payload offset
assert _HDR.size == 64
_DT = {1: np.float32, 2: np.uint8}
_ALIGN = 4096


def _normalise_latent(v):
    t = torch.as_tensor(v).detach().to("cpu", torch.float32)
    if t.dim() == 4 and t.shape[0] == 1:
        t = t[0]
    if t.dim() != 3:
        raise ValueError(f"latent must be (C,H,W) or (1,C,H,W), got {tuple(t.shape)}")
    return t


def _write(path, magic, names, arr, code):
    names_b = json.dumps(list(names)).encode()
    payload = (_HDR.size + len(names_b) + _ALIGN - 1) // _ALIGN * _ALIGN
    d = arr.shape[1:]
    with open(path, "wb") as f:
        f.write(_HDR.pack(magic, arr.shape[0], len(names_b), d[0], d[1], d[2] if len(d) > 2 else 0, code, payload))
        f.write(names_b)
        f.write(b"\0" * (payload - _HDR.size - len(names_b)))
        f.write(np.ascontiguousarray(arr).tobytes())


def _read(path, magic):
    with open(path, "rb") as f:
        m, n, nb, d0, d1, d2, code, payload = _HDR.unpack(f.read(_HDR.size))
        if m != magic:
            raise ValueError(f"{path}: not a {magic.decode()} shard")
        names = json.loads(f.read(nb).decode())
    shape = (n, d0, d1, d2) if d2 else (n, d0, d1)
    if code not in _DT:
        raise ValueError(f"{path}: unknown dtype code {code}")
    arr = np.memmap(path, dtype=_DT[code], mode="r", offset=payload, shape=shape) if n else np.empty(shape, _DT[code])
    if len(names) != n:
        raise ValueError(f"{path}: {len(names)} names for {n} records")
    return names, arr


def write_latent_shard(path, latents):
    """latents: mapping name -> tensor (C,H,W) or (1,C,H,W) (the reference's pickle dict, already loaded)."""
    names = list(latents.keys())
    arr = (torch.stack([_normalise_latent(latents[k]) for k in names]).numpy() if names
           else np.zeros((0, 1, 1, 1), np.float32))
    _write(path, MAGIC_LAT, names, arr, 1)


def read_latent_shard(path):
    """-> (names, memory-mapped fp32 array (N, C, H, W))"""
    return _read(path, MAGIC_LAT)


def _shards(d, ext):
    """Shard files of a directory in part order: numbered parts ({part}.sdlat) numerically, then the rest by name."""
    def key(f):
        stem = os.path.splitext(os.path.basename(f))[0]
        return (0, int(stem), "") if stem.isdigit() else (1, 0, f)
    return sorted(glob.glob(os.path.join(d, "*" + ext)), key=key)


def load_latents(latent_path):
    """Mirror of utils/diffusion_utils.py:7-18 over `*.sdlat` shards: {name: (C, H, W) fp32 tensor}."""
    out = {}
    for fname in _shards(latent_path, ".sdlat"):
        names, arr = read_latent_shard(fname)
        for i, k in enumerate(names):
            out[k] = torch.from_numpy(np.array(arr[i]))
    return out


def class_map_from_png_array(mask_im, mask_h, mask_w, mask_channels):
    """The class map of dataset/celeb_dataset.py:162-171 before its one-hot: nearest resize to (mask_h, mask_w)
    (F.interpolate default, src = floor(dst * in / out)) and clamp(0, mask_channels); -> uint8 (mask_h, mask_w)."""
    a = torch.as_tensor(np.asarray(mask_im, dtype=np.int64))
    if a.dim() != 2:
        raise ValueError("class PNG must be single-channel")
    r = torch.nn.functional.interpolate(a[None, None].float(), size=(mask_h, mask_w), mode="nearest")[0, 0].long()
    return r.clamp(0, mask_channels).to(torch.uint8)


def one_hot_from_class_map(cmap, mask_channels):
    """(…, MH, MW) uint8 -> (…, mask_channels, MH, MW) fp32: the reference's mask tensor (celeb_dataset.py:172-175)."""
    oh = torch.nn.functional.one_hot(cmap.long().clamp(0, mask_channels), mask_channels + 1).movedim(-1, -3)
    return oh[..., 1:, :, :].float()


def write_mask_shard(path, class_maps):
    """class_maps: mapping name -> uint8 (MH, MW) class map (values in [0, mask_channels])."""
    names = list(class_maps.keys())
    arr = (torch.stack([torch.as_tensor(class_maps[k]).to(torch.uint8) for k in names]).numpy() if names
           else np.zeros((0, 1, 1), np.uint8))
    _write(path, MAGIC_MSK, names, arr, 2)


def read_mask_shard(path):
    """-> (names, memory-mapped uint8 array (N, MH, MW))"""
    return _read(path, MAGIC_MSK)


def generate_latents(encode, images, names, latent_dir, shard_size=1000, batch_size=32, device=None):
    """gen_vqvae_latents.py:89-106 as a batched pipeline: encode every image with `encode` (a VQVAE module's
    `encode` -- models.vqvae.VQVAE on the HIP path -- or any callable (B, C, H, W) -> (z, ...) / z) batch_size images
    at a time, and write the quantised latents as `{part}.sdlat` shards of `shard_size` records in image order (the
    reference pickles `{image path: (1, C, h, w)}` every 1000 images as `{part}.pkl`). `images`: a (N, C, H, W)
    tensor (host or device) or a sequence of (C, H, W) / (1, C, H, W) tensors; each batch is moved to `device` before
    `encode` sees it (default: the device of the encoder's module when `encode` is a bound module method, else left
    where it is), so host data-loader images feed the HIP VQVAE directly. Returns the shard paths."""
    if device is None:
        owner = getattr(encode, "__self__", None)
        if isinstance(owner, torch.nn.Module):
            p = next(owner.parameters(), None)
            device = p.device if p is not None else None
    if len(images) != len(names):
        raise ValueError(f"{len(images)} images for {len(names)} names")
    os.makedirs(latent_dir, exist_ok=True)
    paths, part, pending = [], 0, {}

    def flush():
        nonlocal part, pending
        path = os.path.join(latent_dir, f"{part}.sdlat")
        write_latent_shard(path, pending)
        paths.append(path)
        part += 1
        pending = {}

    for s in range(0, len(names), batch_size):
        chunk = images[s:s + batch_size]
        if not isinstance(chunk, torch.Tensor):
            chunk = torch.stack([c[0] if c.dim() == 4 else c for c in chunk])
        if device is not None:
            chunk = chunk.to(device, non_blocking=True)
        with torch.no_grad():
            z = encode(chunk)
        z = (z[0] if isinstance(z, (tuple, list)) else z).detach().to("cpu", torch.float32)
        for i in range(z.shape[0]):
            pending[names[s + i]] = z[i]
            if len(pending) == shard_size:
                flush()
    if pending:
        flush()
    return paths


class ResidentLatentSet:
    """Every latent (and class map) of the training set resident in HBM; `batch(idx)` gathers rows on device.

    Ordering follows `names` (the dataset's image list, celeb_dataset.py:136-153 looks latents up by path and
    then by basename -- the same lookup is applied here)."""

    def __init__(self, latent_dir, names=None, mask_dir=None, device="cuda"):
        table = {}
        for fname in _shards(latent_dir, ".sdlat"):
            ns, arr = read_latent_shard(fname)
            for i, k in enumerate(ns):
                table[k] = (arr, i)
        names = list(table.keys()) if names is None else list(names)

        def find(tab, k):
            if k in tab:
                return tab[k]
            b = os.path.basename(k)
            if b in tab:
                return tab[b]
            raise KeyError(f"no record for {k}")

        first = find(table, names[0])[0]
        lat = torch.empty((len(names),) + tuple(first.shape[1:]), dtype=torch.float32, pin_memory=False)
        for j, k in enumerate(names):
            arr, i = find(table, k)
            lat[j] = torch.from_numpy(np.array(arr[i]))
        self.names = names
        self.latents = lat.to(device)
        self.class_maps = None
        if mask_dir is not None:
            mt = {}
            for fname in _shards(mask_dir, ".sdmsk"):
                ns, arr = read_mask_shard(fname)
                for i, k in enumerate(ns):
                    mt[k] = (arr, i)
            a0 = find(mt, names[0])[0]
            cm = torch.empty((len(names),) + tuple(a0.shape[1:]), dtype=torch.uint8)
            for j, k in enumerate(names):
                arr, i = find(mt, k)
                cm[j] = torch.from_numpy(np.array(arr[i]))
            self.class_maps = cm.to(device)

    def __len__(self):
        return len(self.names)

    def batch(self, idx):
        """idx: int64 device tensor (B,) -> (latents (B, C, H, W) fp32, class maps (B, MH, MW) uint8 or None)."""
        x = self.latents.index_select(0, idx)
        m = self.class_maps.index_select(0, idx) if self.class_maps is not None else None
        return x, m
