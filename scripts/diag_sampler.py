import sys, os
sys.path[:0] = ["stablediffusion-pytorch_amd", "."]
import torch
from safetensors.torch import load_file
from scheduler.linear_noise_scheduler import LinearNoiseScheduler
f = load_file("tests/golden/scheduler_cond.safetensors")
s = LinearNoiseScheduler(1000, 0.00085, 0.012)
for k in ("betas", "alphas", "alpha_cum_prod", "sqrt_alpha_cum_prod", "sqrt_one_minus_alpha_cum_prod"):
    setattr(s, k, f[k])
s._dev = {}
xt, eps, z = f["xt"].cuda(), (f["eps"] * 0.9).cuda(), f["z"].cuda()
prev, x0 = s.sample_prev_timestep(xt, eps, 500, z=z)
t = 500
# torch GPU ops, reference order
tb = {k: getattr(s, k).cuda() for k in ("betas", "alphas", "alpha_cum_prod", "sqrt_one_minus_alpha_cum_prod")}
rx0 = ((xt - (tb["sqrt_one_minus_alpha_cum_prod"][t] * eps)) / torch.sqrt(tb["alpha_cum_prod"][t])).clamp(-1, 1)
mean = xt - ((tb["betas"][t]) * eps) / (tb["sqrt_one_minus_alpha_cum_prod"][t])
mean = mean / torch.sqrt(tb["alphas"][t])
var = (1 - tb["alpha_cum_prod"][t - 1]) / (1.0 - tb["alpha_cum_prod"][t]) * tb["betas"][t]
rprev = mean + var ** 0.5 * z
print("eps*0.9 same?", torch.equal((f["eps"]*0.9), (f["eps"]*0.9)))
for name, a, b in (("x0 vs golden", x0.cpu(), f["x0hat_500"]), ("prev vs golden", prev.cpu(), f["prev_500"]),
                   ("torchgpu x0 vs golden", rx0.cpu(), f["x0hat_500"]), ("torchgpu prev vs golden", rprev.cpu(), f["prev_500"]),
                   ("kernel prev vs torchgpu", prev.cpu(), rprev.cpu())):
    d = (a != b).sum().item()
    print(name, "mismatches", d, "maxabs", (a - b).abs().max().item())
# CPU recompute with same ops
c = {k: getattr(s, k) for k in ("betas", "alphas", "alpha_cum_prod", "sqrt_one_minus_alpha_cum_prod")}
x, e, zz = f["xt"], f["eps"] * 0.9, f["z"]
cm = x - ((c["betas"][t]) * e) / (c["sqrt_one_minus_alpha_cum_prod"][t]); cm = cm / torch.sqrt(c["alphas"][t])
cv = (1 - c["alpha_cum_prod"][t - 1]) / (1.0 - c["alpha_cum_prod"][t]) * c["betas"][t]
cp = cm + cv ** 0.5 * zz
print("cpu recompute prev vs golden", (cp != f["prev_500"]).sum().item())
print("mean cpu vs gpu", (cm != mean.cpu()).sum().item(), "sigma", (cv**0.5).item(), (var**0.5).item())
from safetensors.torch import save_file
os.makedirs("gpurun_out", exist_ok=True)
save_file({"x0": x0.cpu().contiguous(), "prev": prev.cpu().contiguous(), "tx0": rx0.cpu().contiguous()}, "gpurun_out/diag_sampler.safetensors")
