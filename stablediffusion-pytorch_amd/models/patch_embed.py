"""Drop-in mirror of the reference's models/patch_embed.py.

get_patch_position_embedding is the reference's 2-D sin/cos table (patch_embed.py:5-34) as a host-side
API; PatchEmbedding (:37-96) holds the patch Linear with the reference's initialisation. Inside the DIT
the patchify + Linear + position add is ONE implicit-GEMM launch (sdmi.dit_engine); on its own it runs
patch_embed.py:75-96 with the Linear on the HIP leaf path (sdmi.leaf)."""
import torch
import torch.nn as nn

from sdmi import leaf as LF


def get_patch_position_embedding(pos_emb_dim, grid_size, device):
    assert pos_emb_dim % 4 == 0, "Position embedding dimension must be divisible by 4"
    gh, gw = grid_size
    gy, gx = torch.meshgrid(torch.arange(gh, dtype=torch.float32, device=device),
                            torch.arange(gw, dtype=torch.float32, device=device), indexing="ij")
    gy, gx = gy.reshape(-1), gx.reshape(-1)
    q = pos_emb_dim // 4
    factor = 10000 ** (torch.arange(0, q, dtype=torch.float32, device=device) / q)
    ey, ex = gy[:, None].repeat(1, q) / factor, gx[:, None].repeat(1, q) / factor
    return torch.cat([torch.sin(ey), torch.cos(ey), torch.sin(ex), torch.cos(ex)], dim=-1)


class PatchEmbedding(nn.Module):
    def __init__(self, image_height, image_width, im_channels, patch_height, patch_width, hidden_size):
        super().__init__()
        self.image_height = image_height
        self.image_width = image_width
        self.im_channels = im_channels
        self.hidden_size = hidden_size
        self.patch_height = patch_height
        self.patch_width = patch_width
        patch_dim = im_channels * patch_height * patch_width
        self.patch_embed = nn.Sequential(nn.Linear(patch_dim, hidden_size))
        nn.init.xavier_uniform_(self.patch_embed[0].weight)
        nn.init.constant_(self.patch_embed[0].bias, 0)

    def forward(self, x):
        B, C, H, W = x.shape
        ph, pw = self.patch_height, self.patch_width
        assert H % ph == 0, "Input height must be divisible by patch height"
        assert W % pw == 0, "Input width must be divisible by patch width"
        nh, nw = H // ph, W // pw
        # 'b c (nh ph) (nw pw) -> b (nh nw) (ph pw c)'
        tok = x.reshape(B, C, nh, ph, nw, pw).permute(0, 2, 4, 3, 5, 1).reshape(B, nh * nw, ph * pw * C)
        out = LF.call(self.patch_embed, tok)
        return out + get_patch_position_embedding(self.hidden_size, (nh, nw), x.device).to(out.dtype)
