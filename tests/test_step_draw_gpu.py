"""sdmi_step_draw: every random draw of a training step in one launch (CapturedTrainStep._draw; reference
train_ddpm_cond_celebhq_multi_gpu.py:299-330, diffusion_utils.py:21-37). Distribution and semantics checks; the
values are a different random stream from torch's, so they are checked statistically, plus exact determinism."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "stablediffusion-pytorch_amd"))

pytestmark = pytest.mark.gpu


def _draw(noise, t, text, empty, txt, keep, seed, off, T=1000, p_text=0.1, p_keep=0.1):
    from sdmi import _lib
    B = t.numel()
    _lib.check(_lib.lib().sdmi_step_draw(
        noise.data_ptr(), noise.numel(), t.data_ptr(), B, T, text.data_ptr() if txt is not None else None,
        empty.data_ptr() if txt is not None else None, txt.data_ptr() if txt is not None else None,
        empty.numel() if txt is not None else 0, p_text, keep.data_ptr() if keep is not None else None, p_keep,
        seed, off, torch.cuda.current_stream().cuda_stream), "sdmi_step_draw")


def test_step_draw_distribution_and_cond_drop():
    dev = "cuda"
    B = 4096  # many samples: the per-sample rates are checked statistically
    noise = torch.empty(B, 4, 8, 8, device=dev)
    t = torch.empty(B, dtype=torch.long, device=dev)
    text = torch.randn(B, 3, 8, device=dev)
    empty = torch.full((1, 3, 8), 7.0, device=dev)
    txt = torch.empty_like(text)
    keep = torch.empty(B, device=dev)
    _draw(noise, t, text, empty, txt, keep, 1234, 0)
    torch.cuda.synchronize()
    z = noise.flatten()
    assert abs(z.mean().item()) < 0.01 and abs(z.std().item() - 1.0) < 0.01
    assert abs((z.abs() < 1.0).float().mean().item() - 0.6827) < 0.005  # normal, not just unit variance
    assert t.min().item() >= 0 and t.max().item() <= 999 and t.unique().numel() > 900
    dropped = (txt == empty).all(dim=(1, 2))
    kept = (txt == text).all(dim=(1, 2))
    assert bool((dropped | kept).all())  # every text row is either the empty context or the sample's own
    assert abs(dropped.float().mean().item() - 0.1) < 0.02
    assert set(keep.unique().tolist()) <= {0.0, 1.0} and abs(keep.mean().item() - 0.9) < 0.02
    # deterministic for (seed, offset); a new offset draws fresh values; no text / keep buffers is allowed
    n2, t2, txt2, k2 = torch.empty_like(noise), torch.empty_like(t), torch.empty_like(txt), torch.empty_like(keep)
    _draw(n2, t2, text, empty, txt2, k2, 1234, 0)
    assert torch.equal(n2, noise) and torch.equal(t2, t) and torch.equal(txt2, txt) and torch.equal(k2, keep)
    _draw(n2, t2, text, empty, None, None, 1234, 1)
    torch.cuda.synchronize()
    assert not torch.equal(n2, noise) and not torch.equal(t2, t)
    assert torch.equal(txt2, txt) and torch.equal(k2, keep)
