"""Two data-parallel ranks (gloo, both on cuda:0: the one-GPU rehearsal of the N > 1 path) running the cond-UNet
trainer steps with the bf16 gradient wire, so a rocprofv3 kernel trace shows which kernels the exchange adds.
Run it with STEPS=1 and STEPS=3 under `rocprofv3 --kernel-trace`: the difference of the two traces' kernel counts is
the per-step work -- it must contain no aten (at::) kernel (the cast / widen are sdmi_cast_bf16 /
sdmi_widen_bf16_sumsq). Usage: python scripts/wire_rehearsal.py <steps> [fp32|bf16]"""
import os
import socket
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "stablediffusion-pytorch_amd"), REPO]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, steps, wire):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import sd_oracle as O
    from tests.golden.configs import SMALL_COND
    from sdmi.trainer import DDPMTrainer
    sd = O.deterministic_state(O.unet_param_shapes(SMALL_COND), seed=3)
    tr = DDPMTrainer(SMALL_COND, sd, "cuda", group=dist.group.WORLD, grad_wire=wire, bucket_bytes=1 << 20)
    g = torch.Generator().manual_seed(40 + rank)
    B = 2
    x0, noise = torch.randn(B, 4, 32, 32, generator=g).cuda(), torch.randn(B, 4, 32, 32, generator=g).cuda()
    t = torch.randint(0, 1000, (B,), generator=g).cuda()
    text = torch.randn(B, 77, 64, generator=g).cuda()
    mask = torch.nn.functional.one_hot(torch.randint(0, 19, (B, 64, 64), generator=g), 19).movedim(-1, 1)[:, 1:]
    mask = mask.float().contiguous().cuda()
    torch.cuda.synchronize()
    for _ in range(steps):
        tr.step(x0, noise, t, text, mask)
    tr.sync_optimizer()
    torch.cuda.synchronize()
    if rank == 0:
        print(f"rank 0: {steps} steps, wire {tr.grad_wire}, buckets {tr.reducer.nb}, loss {tr.state[6].item():.5f}, "
              f"norm {tr.state[0].item():.5f}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    wire = sys.argv[2] if len(sys.argv) > 2 else "bf16"
    mp.spawn(worker, args=(2, _port(), steps, wire), nprocs=2, join=True)
