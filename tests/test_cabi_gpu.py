"""The C ABI called from C (no PyTorch, no C++): tests/cabi/cabi_check.c -- built by __graft_entry__.build() with gcc
against include/sdmi.h and libsdmi.so -- runs a 3x3 convolution through sdmi_gemm_plan + sdmi_gemm (implicit GEMM,
models/blocks.py:48-53) and a cross-attention core through sdmi_attn_fwd (models/blocks.py:140) on its own device
buffers and writes inputs and outputs to files; this test recomputes both in torch fp32 from the same bf16 inputs.
Tolerances: bf16 outputs of fp32 accumulations -- max |diff| <= 2e-2 * max |ref| (conv), <= 2e-2 (attention,
|o| <= max |v| = 1); base-2 log-sum-exp within 1e-3 relative."""
import os
import subprocess

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cabi", "cabi_check")


def _load(d, name, shape):
    raw = np.fromfile(os.path.join(d, name), dtype=np.uint16 if name.endswith(".bf16") else np.float32)
    t = torch.from_numpy(raw.astype(np.int32) if name.endswith(".bf16") else raw)
    if name.endswith(".bf16"):
        t = (t.to(torch.int32) << 16).view(torch.float32)
    return t.reshape(shape)


def test_c_caller_conv_and_attention(tmp_path):
    assert os.path.exists(BIN), "tests/cabi/cabi_check missing: run __graft_entry__.build() first"
    r = subprocess.run([BIN, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    B, H, W, Cin, Cout = 2, 16, 16, 64, 128
    x = _load(tmp_path, "conv_x.bf16", (B, H, W, Cin)).permute(0, 3, 1, 2)
    w = _load(tmp_path, "conv_w.bf16", (Cout, 3, 3, Cin)).permute(0, 3, 1, 2)
    b = _load(tmp_path, "conv_b.f32", (Cout,))
    y = _load(tmp_path, "conv_y.bf16", (B, H, W, Cout)).permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(x, w, b, padding=1)
    assert (y - ref).abs().max().item() <= 2e-2 * ref.abs().max().item(), (y - ref).abs().max().item()
    N, S, heads, hd = 256, 77, 4, 32
    C = heads * hd
    q = _load(tmp_path, "attn_q.bf16", (B, N, heads, hd)).transpose(1, 2)
    k = _load(tmp_path, "attn_k.bf16", (B, S, heads, hd)).transpose(1, 2)
    v = _load(tmp_path, "attn_v.bf16", (B, S, heads, hd)).transpose(1, 2)
    o = _load(tmp_path, "attn_o.bf16", (B, N, heads, hd)).transpose(1, 2)
    lse = _load(tmp_path, "attn_lse.f32", (B, heads, N))
    s = (q / hd ** 0.5) @ k.transpose(-1, -2)
    ref_o = torch.softmax(s, -1) @ v
    assert (o - ref_o).abs().max().item() <= 2e-2, (o - ref_o).abs().max().item()
    # lse is base 2 (include/sdmi.h): log2 sum_j 2^(s_ij log2 e) = ln-LSE x log2 e
    ref_lse = torch.logsumexp(s, -1)
    err = (lse * np.log(2.0) - ref_lse).abs().max().item()
    assert err <= 1e-3 * max(1.0, ref_lse.abs().max().item()), err
