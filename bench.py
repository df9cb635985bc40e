"""Benchmark: DDPM train steps/sec of the conditional UNet (config/celebhq_text_image_cond.py, CelebHQ-256
latents (B,4,32,32), per-GPU batch 32, text (B,77,512) + mask (B,18,512,512) conditioning) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
    (N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N)

One step = the reference's training step (train_ddpm_cond_celebhq_multi_gpu.py:299-378) on a synthetic
batch already resident in HBM: cond-drop, noise/t draw, add_noise, forward, MSE, backward, RCCL
all-reduce (N > 1), clip(1.0), Adam(1e-5), EMA(0.9999), bf16 weight repack. Prints ONE JSON line.
"""
import argparse
import json
import re
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "stablediffusion-pytorch_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "DDPM train steps/sec (cond-UNet, CelebHQ-256 latents, B=32) at 1/2/4/8 MI355X"
FLOP_PER_STEP = 3.8815e12      # cond-UNet fwd+bwd at B=32 (FlopCounterMode on the oracle)
# secondary workloads (--workload): DiT-12L training step (fwd+bwd 6.759e11 FLOP at B=32)
WORKLOADS = {
    "cond-unet": dict(metric=METRIC, flop=FLOP_PER_STEP),
    "dit": dict(metric="DDPM train steps/sec (DiT-12L image-cond, CelebHQ-256 latents, B=32) on MI355X", flop=6.759e11),
    # BASELINE config 3: config/celebhq.yaml unconditional UNet (tools/train_ddpm_vqvae.py step: Adam, no clip / EMA)
    "uncond-unet": dict(metric="DDPM train steps/sec (uncond-UNet celebhq.yaml, CelebHQ-256 latents, B=32) on MI355X",
                        flop=3.4814e12),
    # VQVAE encode + decode (no grad) of a batch of 8 CelebHQ-256 images: 2.9497e11 FLOP per image
    "vqvae": dict(metric="VQVAE encode+decode steps/sec (celebhq.yaml autoencoder, 256x256, B=8) on MI355X",
                  flop=8 * 2.9497e11),
    # VQVAE generator training step (train_vqvae_celebhq.py:405-466 without LPIPS / GAN): fwd + bwd ~ 3x the forward
    "vqvae-train": dict(metric="VQVAE train steps/sec (celebhq autoencoder, 256x256, B=8, recon + codebook + "
                               "commitment, Adam) on MI355X", flop=3 * 8 * 2.9497e11),
    # DDPM sampling (tools/sample_ddpm_text_image_cond.py loop, train_num_samples = 1 in the reference config):
    # one step = cond-UNet forward at batch --sample-batch + the reverse step; fwd 1.2988e12 FLOP at B=32
    "sample": dict(metric="DDPM sampling steps/sec (cond-UNet, CelebHQ-256 latents, captured loop) on MI355X",
                   flop=1.2988e12 / 32),
}
PEAK_BF16 = 2.5e15             # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM = 8.0e12


# GEMM mode tag -> kernel symbol (gemm.hip): the launch's mainloop variant (as the library reports it after its own
# downgrades, sdmi_gemm_kernel_info) -> the template arguments of its instantiation
#   gemm_dma_kernel<AM, BMODE, STAGES, TBN, TBM, NWN, RED, KBK, GNE, KG>  (RED / GNE: '*', one name for all of them)
DMA_VARIANTS = {2: (2, None, 128, 2, 64, 1), 3: (3, 128, 128, 2, 64, 1), 4: (4, None, 128, 4, 32, 1),
                5: (3, None, 128, 2, 32, 1), 6: (4, 128, 128, 2, 64, 1), 7: (6, 64, 64, 4, 64, 1),
                8: (6, 128, 64, 4, 64, 1), 9: (3, 128, 64, 4, 64, 1), 10: (2, 128, 64, 4, 64, 1),
                11: (2, 128, 128, 2, 64, 2)}


def kernel_name(tag, info):
    """Kernel instantiation of a profiled sdmi_gemm launch as a glob over rocprofv3's demangled names, from its mode
    tag (gemm_a<A>b<B>) and the variant / tile_n the library reported."""
    a, b = re.match(r"gemm_a(\d)b(\d)", tag).groups()
    v = int(re.search(r"variant=(\d+)", info).group(1))
    tn = int(re.search(r"tile_n=(\d+)", info).group(1))
    if v == 0:
        return f"gemm_kernel<{a}, {b}, *>"
    st, tbn, tbm, nwn, kbk, kg = DMA_VARIANTS[v]
    return f"gemm_dma_kernel<{a}, {b}, {st}, {tbn or tn}, {tbm}, {nwn}, *, {kbk}, *, {kg}>"


def kernel_matches(pattern, name):
    """rocprofv3 kernel name (demangled, possibly with 'void (anonymous namespace)::' and an argument list) vs a
    kernel_name() glob"""
    import fnmatch
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").strip()
    n = n[:n.index(">(") + 1] if ">(" in n else n
    return fnmatch.fnmatchcase(n, pattern)


def _evidence_files(workload, kind):
    """Committed rocprofv3 evidence of `workload` (kind 'pmc_traffic' or 'roofline_evidence'), newest round first:
    profiles/rNN_<workload>_<kind>.json, written by scripts/gpu_profile.sh from the tree whose source digest
    (sdmi._build.source_digest) each file records."""
    import glob
    wl = workload.replace("-", "_")
    return sorted(glob.glob(os.path.join(REPO, "profiles", f"r[0-9]*_{wl}_{kind}.json")), reverse=True)


def _load_evidence(workload, kind, digest):
    """(table, file name, digest matches the running tree) of the newest evidence file measured on THIS tree, else of
    the newest one at all (flagged stale), else (None, None, False)."""
    files = _evidence_files(workload, kind)
    loaded = []
    for f in files:
        try:
            loaded.append((json.load(open(f)), f))
        except (OSError, ValueError):
            continue
    for d, f in loaded:
        if d.get("_meta", {}).get("source_digest") == digest:
            return d, os.path.basename(f), True
    if loaded:
        return loaded[0][0], os.path.basename(loaded[0][1]), False
    return None, None, False


def pmc_traffic(workload, kernel, unsplit):
    """HBM bytes per launch of `kernel` (read x2-corrected FETCH_SIZE + WRITE_SIZE) from the committed rocprofv3 --pmc
    passes of this same bench command: the roofline-evidence file (scripts/roofline_evidence.py: exactly the launches
    the bench times -- unsplit ones, or all) when it names this kernel and launch set, else the per-kernel table
    (scripts/pmc_summary.py, all launches). Returns (bytes or None, provenance dict)."""
    from sdmi._build import source_digest
    digest = source_digest()
    ev, ev_file, ev_ok = _load_evidence(workload, "roofline_evidence", digest)
    launches = "unsplit" if unsplit else "all"
    if ev and ev.get("kernel") == kernel and ev.get("launches") == launches and ev.get("traffic_bytes_per_launch"):
        return ev["traffic_bytes_per_launch"], {
            "file": ev_file, "tree_digest": digest, "measured_on_this_tree": ev_ok,
            "unit": f"bytes/launch (HBM, PMC FETCH_SIZE x2 + WRITE_SIZE, the kernel's {launches} launches: the ones "
                    "timed here)", "trace_avg_us": ev.get("trace_avg_us")}
    table, t_file, t_ok = _load_evidence(workload, "pmc_traffic", digest)
    if table:
        # the kernel_name() glob covers several instantiations (RED / GNE): their launch-weighted average
        keys = [k for k in table if k != "_meta" and kernel_matches(kernel, k)]
        n = sum(table[k]["launches"] for k in keys)
        if n:
            b = sum((table[k]["read_bytes_per_launch"] + table[k]["write_bytes_per_launch"]) * table[k]["launches"]
                    for k in keys) / n
            return b, {"file": t_file, "tree_digest": digest, "measured_on_this_tree": t_ok,
                       "unit": "bytes/launch (HBM, PMC FETCH_SIZE x2 + WRITE_SIZE, all launches of the kernel)",
                       "instantiations": keys}
    return None, {"file": None, "tree_digest": digest, "measured_on_this_tree": False}


def uncond_config():
    from tests.golden.configs import full_uncond_config
    return full_uncond_config()


def cond_config():
    from tests.golden.configs import full_cond_config
    return full_cond_config()


def synthetic_batch(B, device, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x0 = torch.randn(B, 4, 32, 32, generator=g)
    text = torch.randn(B, 77, 512, generator=g)
    empty = torch.randn(1, 77, 512, generator=g)  # stand-in for the CLIP embedding of "" (text_utils.py)
    cmap = torch.randint(0, 19, (B, 512, 512), generator=g)
    x0, text, empty = x0.to(device), text.to(device), empty.to(device)
    mask = torch.nn.functional.one_hot(cmap.to(device).long(), 19).movedim(-1, 1)[:, 1:].float().contiguous()
    return x0, text, empty, mask


def dit_config():
    from tests.golden.configs import dit12l_config
    return dit12l_config()


def cpu_model():
    """The host CPU as /proc/cpuinfo names it, with its logical CPU count (lscpu's 'Model name' / 'CPU(s)')."""
    name = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                name = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return f"{name}, {os.cpu_count()} logical CPUs visible"


def cpu_threads():
    """Threads for the CPU baseline: the physical cores of this process's CPU affinity set (sibling hyperthreads
    counted once, from /sys/devices/system/cpu/cpu*/topology), capped by the CPU share the host grants this job -- a
    cgroup CPU quota (/sys/fs/cgroup/cpu.max) and the per-GPU thread share the GPU pool exports as OMP_NUM_THREADS
    (16 per GPU: a 1-GPU job must not spread onto the other GPUs' cores). Returns (threads, facts)."""
    aff = sorted(os.sched_getaffinity(0))
    cores = set()
    for c in aff:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            cores.add((open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip()))
        except OSError:
            cores.add(("cpu", c))
    phys = len(cores)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    share = os.environ.get("OMP_NUM_THREADS")
    share = int(share) if share and share.isdigit() and int(share) > 0 else None
    threads = phys
    for cap in (quota, share):
        if cap is not None:
            threads = min(threads, max(1, int(cap)))
    return threads, {"affinity_logical_cpus": len(aff), "affinity_physical_cores": phys, "cgroup_cpu_quota": quota,
                     "omp_num_threads_share": share}


def timed_cpu(fn, warmup=1, timed=3):
    """Median wall time of `timed` calls of fn after `warmup` calls (1 warm-up + 3 timed)."""
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(timed):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2], ts


def _cpu_result(per, ts, threads, what):
    return dict(value=1.0 / per, unit="steps/s", cores=threads, kind="port", cpu=cpu_model(), host=cpu_threads()[1],
                sample=f"{what}; median of {len(ts)} timed steps {per:.2f} s/step (all: "
                       f"{', '.join(f'{t:.2f}' for t in ts)}), torch CPU {torch.__version__} with {threads} threads")


def gemm_roofline(prof, PROF_STEPS, workload):
    """Dominant-kernel roofline from PROF_STEPS profiled steps' sdmi GEMM launches (K.PROFILE records: HIP events on
    the launch's own stream): the kernel instantiation with the largest event time, its achieved TFLOP/s over its
    unsplit launches (or all of them, each then including its split-K reducer), algorithmic bytes per launch, and the
    HBM traffic per launch from the committed rocprofv3 --pmc evidence of this workload."""
    by, per_kernel = {}, {}
    for tag, fl, e0, e1, sp in prof:
        if not tag.startswith("gemm"):
            continue
        ms = e0.elapsed_time(e1)
        a = by.setdefault(tag, [0.0, 0.0, 0])
        a[0] += fl
        a[1] += ms
        a[2] += 1
        kern = kernel_name(tag, sp)
        split = int(re.search(r"splits=(\d+)", sp).group(1)) > 1
        k = per_kernel.setdefault(kern, {"fl": 0.0, "ms": 0.0, "n": 0, "fl1": 0.0, "ms1": 0.0, "n1": 0, "mode": tag,
                                         "by": 0.0, "by1": 0.0})
        nb = re.search(r"bytes=(\d+)", sp)
        nb = float(nb.group(1)) if nb else 0.0
        k["fl"] += fl
        k["ms"] += ms
        k["n"] += 1
        k["by"] += nb
        if not split:  # the event brackets the kernel alone (split launches add a reducer launch)
            k["fl1"] += fl
            k["ms1"] += ms
            k["n1"] += 1
            k["by1"] += nb
    tot_fl = sum(v[0] for v in by.values())
    tot_ms = sum(v[1] for v in by.values())
    dname, d = max(per_kernel.items(), key=lambda kv: kv[1]["ms"])
    # the unsplit launches (events bracket the kernel alone) represent the kernel when they carry most of its work;
    # otherwise (e.g. DiT weight gradients, whose few unsplit launches are the tiny t-emb GEMMs) all launches count,
    # each event then including its split-K reducer (a lower bound on the kernel's own rate)
    use1 = d["n1"] > 0 and d["fl1"] >= 0.5 * d["fl"]
    dfl, dms, dn, dby = (d["fl1"], d["ms1"], d["n1"], d["by1"]) if use1 else (d["fl"], d["ms"], d["n"], d["by"])
    traffic, traffic_src = pmc_traffic(workload, dname, use1)
    algo = dby / dn if dn else None  # algorithmic bytes per launch (sdmi.kernels.algo_bytes over the same launches)
    return {"kernel_id": dname, "launch_set": "unsplit" if use1 else "all",
            "bound": "mfma", "kernel": f"sdmi {dname} ({d['mode']}: implicit-GEMM conv fwd/dgrad)"
            if d["mode"] == "gemm_a1b0" else f"sdmi {dname} ({d['mode']})",
            "achieved": dfl / (dms * 1e-3) / 1e12, "peak": PEAK_BF16 / 1e12, "unit": "TFLOP/s",
            "frac": dfl / (dms * 1e-3) / PEAK_BF16, "traffic": traffic,
            "traffic_unit": traffic_src.get("unit"), "traffic_source": traffic_src,
            "algorithmic_bytes": algo,
            "algorithmic_bytes_note": "per launch: unique operand bytes at their dtypes (conv im2col = the gathered "
                                      "activation), output and fused epilogue reads, averaged over the same launches",
            "traffic_ratio": traffic / algo if traffic and algo else None,
            "launches": dn // PROF_STEPS,
            "launches_note": f"unsplit launches of the kernel per step (HIP events on its stream, {PROF_STEPS} "
                             "profiled steps averaged)" if use1 else "all launches (each includes its split-K reducer)",
            "avg_launch_us": dms * 1e3 / dn, "flop_per_launch": dfl / dn,
            "kernel_ms_per_step": d["ms"] / PROF_STEPS, "kernel_launches_per_step": d["n"] // PROF_STEPS,
            "all_gemm": {"tflops": tot_fl / (tot_ms * 1e-3) / 1e12, "ms_per_step": tot_ms / PROF_STEPS,
                         "launches": sum(v[2] for v in by.values()) // PROF_STEPS},
            "per_mode": {k: {"tflops": v[0] / (v[1] * 1e-3) / 1e12, "ms": v[1] / PROF_STEPS,
                             "launches": v[2] // PROF_STEPS} for k, v in by.items()},
            "per_kernel": {k: {"tflops": v["fl"] / (v["ms"] * 1e-3) / 1e12, "ms": v["ms"] / PROF_STEPS,
                               "launches": v["n"] // PROF_STEPS} for k, v in per_kernel.items()}}


def cpu_baseline_dit(cfg, B=32):
    """The DiT oracle's fp32 training step (Model_DiT_12L_train.py:300-375) on the host cores."""
    from oracle import sd_oracle as O, dit_oracle as DO
    threads, _ = cpu_threads()
    torch.set_num_threads(threads)
    sd = O.deterministic_state(DO.dit_param_shapes(cfg), seed=0)
    opt = O.AdamState(sd)
    sched = O.SchedulerTables(1000, 0.00085, 0.012)
    g = torch.Generator().manual_seed(1111)
    x0 = torch.randn(B, 4, 32, 32, generator=g)
    cmap = torch.randint(0, 19, (B, 512, 512), generator=g)
    mask = torch.nn.functional.one_hot(cmap, 19).movedim(-1, 1)[:, 1:].float()

    def step():
        noise = torch.randn(x0.shape, generator=g)
        t = torch.randint(0, 1000, (B,), generator=g)
        DO.dit_train_step(sd, opt, cfg, sched, x0, noise, t, {"image": mask})
    per, ts = timed_cpu(step)
    return _cpu_result(per, ts, threads, f"DiT oracle fp32 train step (fwd+bwd+clip+Adam), B={B}, 1 warm-up")


def vqvae_config():
    from tests.golden.configs import vqvae_celebhq_config
    return vqvae_celebhq_config()


def cpu_baseline_vqvae(cfg, B=8):
    """The VQVAE oracle's fp32 encode + decode on the host cores."""
    from oracle import sd_oracle as O, vqvae_oracle as VO
    threads, _ = cpu_threads()
    torch.set_num_threads(threads)
    sd = O.deterministic_state(VO.vqvae_param_shapes(cfg), seed=0)
    x = torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(1111)) * 2 - 1

    def step():
        with torch.no_grad():
            zq, _, _ = VO.encode(sd, cfg, x)
            VO.decode(sd, cfg, zq)
    per, ts = timed_cpu(step)
    return _cpu_result(per, ts, threads, f"VQVAE oracle fp32 encode+decode, B={B} at 256x256, 1 warm-up")


def cpu_baseline(cfg, B=32, uncond=False, small_batch=4):
    """The oracle (CPU fp32 restatement of the reference step) on the host cores: B=32 (the bench workload) and
    B=small_batch, each 1 warm-up + 3 timed, median."""
    from oracle import sd_oracle as O
    threads, _ = cpu_threads()
    torch.set_num_threads(threads)
    res = None
    for b in (B, small_batch):
        sd = O.deterministic_state(O.unet_param_shapes(cfg, base="uncond" if uncond else None), seed=0)
        ema = {k: v.clone() for k, v in sd.items()}
        opt = O.AdamState(sd)
        sched = O.SchedulerTables(1000, 0.0015, 0.0195) if uncond else O.SchedulerTables(1000, 0.00085, 0.012)
        g = torch.Generator().manual_seed(1111)
        x0 = torch.randn(b, 4, 32, 32, generator=g)
        text = torch.randn(b, 77, 512, generator=g)
        cmap = torch.randint(0, 19, (b, 512, 512), generator=g)
        mask = torch.nn.functional.one_hot(cmap, 19).movedim(-1, 1)[:, 1:].float()

        def step():
            noise = torch.randn(x0.shape, generator=g)
            t = torch.randint(0, 1000, (b,), generator=g)
            if uncond:  # tools/train_ddpm_vqvae.py: no clip (inf), no EMA (decay 0: a copy, negligible)
                O.train_step(sd, ema, opt, cfg, sched, x0, noise, t, None, lr=5e-6, clip=float("inf"), ema_decay=0.0)
            else:
                O.train_step(sd, ema, opt, cfg, sched, x0, noise, t, {"text": text, "image": mask})
        per, ts = timed_cpu(step)
        what = "fwd+bwd+Adam" if uncond else "fwd+bwd+clip+Adam+EMA"
        r = _cpu_result(per, ts, threads, f"oracle fp32 train step ({what}), B={b}, 1 warm-up")
        if res is None:
            res = r
        else:
            res[f"b{b}"] = {"value": r["value"], "unit": "steps/s", "sample": r["sample"]}
    return res


def main_vqvae(args, wl, world, rank, device):
    """VQVAE encode + decode (inference) of a synthetic CelebHQ-256 batch of 8 images per GPU (replicas)."""
    from models.vqvae import VQVAE
    cfg = vqvae_config()
    torch.manual_seed(1111)
    model = VQVAE(3, cfg).to(device)
    B = 8
    x = (torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(1111 + rank)) * 2 - 1).to(device)
    eng = model._eng(x)

    def step():
        zq, loss, idx = eng.encode(x)
        eng.decode(zq)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = e.item()
    sps = args.steps / elapsed
    from sdmi import kernels as K
    PROF_STEPS = 3
    K.PROFILE = []
    for _ in range(PROF_STEPS):
        step()
    torch.cuda.synchronize()
    prof, K.PROFILE = K.PROFILE, None
    roof = gemm_roofline(prof, PROF_STEPS, args.workload)
    result = {"metric": wl["metric"], "value": sps * world, "unit": "steps/s", "n_gpus": world, "steps": args.steps,
              "warmup": args.warmup, "ms_per_step": 1000.0 / sps, "higher_is_better": True, "scaling": "weak",
              "vs_baseline": None, "dtype": "bf16", "data": "synthetic 256x256 images, random-init weights",
              "config": {"workload": "VQVAE celebhq.yaml encode + quantize + decode (inference)", "model": "VQVAE 22.0M",
                         "per_gpu_batch": B, "image": [3, 256, 256], "latent": [4, 32, 32],
                         "parallelism": f"replicas{world}"},
              "images_per_s": sps * B * world, "model_flops_utilization": wl["flop"] * sps / PEAK_BF16,
              "roofline": roof}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_vqvae(cfg)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline_vqvae_train(cfg, B=8):
    """The VQVAE oracle's fp32 generator step (train_grads: forward, losses, autograd backward) on the host cores;
    3 timed steps, no warm-up (~11 s each)."""
    from oracle import sd_oracle as O, vqvae_oracle as VO
    threads, _ = cpu_threads()
    torch.set_num_threads(threads)
    sd = O.deterministic_state(VO.vqvae_param_shapes(cfg), seed=0)
    x = torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(1111)) * 2 - 1
    per, ts = timed_cpu(lambda: VO.train_grads(sd, cfg, x), warmup=0)
    return _cpu_result(per, ts, threads, f"VQVAE oracle fp32 fwd + losses + bwd (no optimizer), B={B} at 256x256, "
                                         "no warm-up")


def main_vqvae_train(args, wl, world, rank, device):
    """VQVAE generator training step (sdmi.vqvae_train.VQVAETrainer) on a synthetic CelebHQ-256 batch of 8 images per
    GPU, recorded once and replayed (sdmi.plan); N > 1: data parallel with one bucketed all-reduce per step."""
    from models.vqvae import VQVAE
    from sdmi.plan import StepPlan
    from sdmi.vqvae_train import VQVAETrainer
    cfg = vqvae_config()
    torch.manual_seed(1111)
    init = VQVAE(3, cfg).state_dict()
    B = 8
    x = (torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(1111 + rank)) * 2 - 1).to(device)
    tr = VQVAETrainer(cfg, {k: v.to(device) for k, v in init.items()}, device,
                      group=dist.group.WORLD if world > 1 else None)
    for _ in range(2):
        tr.step(x)
    plan = StepPlan(lambda: tr.step(x), device) if args.issue == "plan" else None
    step = plan.replay if plan is not None else (lambda: tr.step(x))
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = e.item()
    sps = args.steps / elapsed
    losses = tr.losses()
    # dominant-kernel roofline: eager steps with the GEMM launches timed by HIP events on their own streams
    from sdmi import kernels as K
    PROF_STEPS = 3
    K.PROFILE = []
    for _ in range(PROF_STEPS):
        tr.step(x)
    torch.cuda.synchronize()
    prof, K.PROFILE = K.PROFILE, None
    roof = gemm_roofline(prof, PROF_STEPS, args.workload)
    result = {"metric": wl["metric"], "value": sps * world, "unit": "steps/s", "n_gpus": world, "steps": args.steps,
              "warmup": args.warmup, "ms_per_step": 1000.0 / sps, "higher_is_better": True, "scaling": "weak",
              "vs_baseline": None, "dtype": "bf16", "data": "synthetic 256x256 images, random-init weights",
              "config": {"workload": "VQVAE celebhq.yaml generator step: fwd, recon MSE + codebook + commitment, bwd, "
                                     "Adam(2e-5, betas (0.5, 0.999)); LPIPS / GAN out of scope",
                         "model": "VQVAE 22.0M", "per_gpu_batch": B, "image": [3, 256, 256], "latent": [4, 32, 32],
                         "parallelism": f"dp{world}", "issue": args.issue},
              "images_per_s": sps * B * world, "model_flops_utilization": wl["flop"] * sps / PEAK_BF16,
              "last_losses": losses, "roofline": roof}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_vqvae_train(cfg)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_sample(args, wl, world, rank, device):
    """Reverse-diffusion sampling throughput: the cond-UNet sampler loop recorded once and replayed (sdmi.sampling),
    against the same loop issued step by step (eager). Replicas for N > 1 (sampling does not shard)."""
    import models.unet_cond_base as mc
    from scheduler.linear_noise_scheduler import LinearNoiseScheduler
    from sdmi.sampling import DDPMSampleLoop
    cfg = cond_config()
    torch.manual_seed(1111)
    model = mc.Unet(4, cfg).to(device).eval()
    B = args.sample_batch
    x0, text, empty, mask = synthetic_batch(B, device, 1111 + rank)
    sched = LinearNoiseScheduler(1000, 0.00085, 0.012)
    cond = {"text": text, "image": mask}
    xT = torch.randn(B, 4, 32, 32, generator=torch.Generator().manual_seed(5 + rank)).to(device)
    if args.sampler == "ddim":  # DDIMSampler.forward (scheduler :209-256): `--steps` (t, t_prev) pairs, eta 0
        from scheduler.linear_noise_scheduler import DDIMSampler
        from sdmi.sampling import DDIMSampleLoop
        abar = DDIMSampler(model, (0.00085, 0.012), 1000).alpha_t_bar
        loop = DDIMSampleLoop(model, abar, (B, 4, 32, 32), cond_input=cond, steps=args.steps, seed=rank)
        run = lambda n, cap: loop.run(xT, captured=cap)  # noqa: E731  (always the whole `--steps` loop)
    else:
        loop = DDPMSampleLoop(model, sched, (B, 4, 32, 32), cond_input=cond, seed=rank)
        run = lambda n, cap: loop.run(xT, steps=n, captured=cap)  # noqa: E731
    res = {}
    for mode in ("captured", "eager"):
        cap = mode == "captured"
        run(args.warmup + 1, cap)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        run(args.steps, cap)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            e = torch.tensor([el], device=device, dtype=torch.float64)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            el = e.item()
        res[mode] = args.steps / el
    sps = res["captured"]
    # roofline of the step's GEMM launches (every implicit-GEMM conv and linear of the forward, HIP events on their
    # stream, one eager reverse step): at B = 1 the grids are small and each launch is latency-bound
    from sdmi import kernels as K
    K.PROFILE = []
    loop._refresh()
    loop._step()  # one eager reverse step (model forward + the sampler's update kernel)
    torch.cuda.synchronize()
    prof, K.PROFILE = K.PROFILE, None
    gfl = sum(p[1] for p in prof if p[0].startswith("gemm"))
    gms = sum(p[2].elapsed_time(p[3]) for p in prof if p[0].startswith("gemm"))
    ngemm = sum(1 for p in prof if p[0].startswith("gemm"))
    roof = {"bound": "mfma", "kernel": "sdmi gemm (all implicit-GEMM conv / linear launches of one reverse step)",
            "achieved": gfl / (gms * 1e-3) / 1e12 if gms else None, "peak": PEAK_BF16 / 1e12, "unit": "TFLOP/s",
            "frac": gfl / (gms * 1e-3) / PEAK_BF16 if gms else None, "traffic": None, "launches": ngemm,
            "avg_launch_us": gms * 1e3 / max(1, ngemm), "flop_per_launch": gfl / max(1, ngemm),
            "gemm_ms_per_step": gms}
    result = {"metric": wl["metric"].replace("DDPM", "DDIM") if args.sampler == "ddim" else wl["metric"], "value": sps * world, "unit": "steps/s", "n_gpus": world, "steps": args.steps,
              "warmup": args.warmup, "ms_per_step": 1000.0 / sps, "higher_is_better": True, "scaling": "weak",
              "vs_baseline": None, "dtype": "bf16", "data": "synthetic latents / text / masks, random-init weights",
              "config": {"workload": f"cond-UNet {args.sampler.upper()} reverse step (model forward + "
                                     f"{'DDIM update' if args.sampler == 'ddim' else 'sample_prev_timestep'}), captured",
                         "sampler": args.sampler, "issue": loop.issue,
                         "model": "cond-UNet 118.5M", "samples_per_gpu": B, "latent": [4, 32, 32],
                         "parallelism": f"replicas{world}"},
              "eager_steps_per_s": res["eager"], "captured_speedup": sps / res["eager"],
              "model_flops_utilization": wl["flop"] * B * sps / PEAK_BF16, "roofline": roof}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def collective_facts(world, device):
    """N > 1: what the process group itself reports -- backend, its world size, an all-reduce of ones through it (the
    sum proves every rank took part in a collective on this group), and each rank's device (ordinal, PCI bus, uuid),
    so a scaling run shows that RCCL saw N ranks on N distinct GPUs."""
    if world <= 1:
        return None
    one = torch.ones(1, device=device)
    dist.all_reduce(one)
    props = torch.cuda.get_device_properties(device)
    mine = {"rank": dist.get_rank(), "device": device.index, "pci_bus_id": getattr(props, "pci_bus_id", None),
            "pci_domain_id": getattr(props, "pci_domain_id", None), "uuid": str(getattr(props, "uuid", ""))}
    devs = [None] * world
    dist.all_gather_object(devs, mine)
    distinct = len({(d["pci_domain_id"], d["pci_bus_id"], d["uuid"]) for d in devs})
    return {"backend": dist.get_backend(), "rccl_ranks": dist.get_world_size(),
            "allreduce_of_ones": one.item(), "devices": devs, "distinct_devices": distinct}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--sample-batch", type=int, default=1, help="samples per GPU of --workload sample (reference: 1)")
    ap.add_argument("--sampler", default="ddpm", choices=("ddpm", "ddim"),
                    help="--workload sample: DDPM (T steps of sample_prev_timestep) or DDIM (--steps pairs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", default="cond-unet", choices=sorted(WORKLOADS),
                    help="cond-unet (the headline metric, default), uncond-unet (celebhq.yaml), dit (DiT-12L training "
                         "step), vqvae (encode + decode), vqvae-train (VQVAE generator step) or sample (captured DDPM sampling loop)")
    ap.add_argument("--profile-gemm", action="store_true", default=True)
    ap.add_argument("--grad-wire", default=None, choices=("fp32", "bf16"),
                    help="N > 1: gradient all-reduce wire format (default fp32 as the reference's DDP; bf16 halves "
                         "the bytes)")
    ap.add_argument("--force-reducer", action="store_true",
                    help="N = 1 only: run the headline step with the N > 1 gradient path forced on -- an RCCL ('nccl') "
                         "process group of one rank, the bucketed all-reduce reducer on its stream and the per-bucket "
                         "norm blocks (sdmi.reducer) -- and report exchange_tail_ms: the part of the N > 1 step that "
                         "this one-GPU pool can time")
    ap.add_argument("--issue", default="plan", choices=("plan", "eager", "graph"),
                    help="plan (default): the step recorded once and its native calls replayed (sdmi.plan); eager: "
                         "per-step Python issue; graph: single-stream hipGraph (N == 1)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SDMI_BENCH_BACKEND=gloo (rehearsal only): N ranks share the GPUs present (local % device_count) over gloo,
    # so the N > 1 issue / barrier / max-over-ranks path can be exercised on a one-GPU box
    backend = os.environ.get("SDMI_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    # the engines' concurrent streams bound to hardware queues of their own before RCCL binds its streams
    # (sdmi/streams.py: HIP binds a stream to a queue at first use, rotating once all four exist)
    if os.environ.get("SDMI_RESERVE_STREAMS", "1") == "1":
        from sdmi import streams
        streams.reserve(device, n=streams.workload_streams(args.workload, world))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    collectives = collective_facts(world, device)
    forced = args.force_reducer and world == 1
    if forced:  # an RCCL group of one rank: the reducer's all-reduces are identities, their cost is real
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(sk.getsockname()[1]))
        sk.close()
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=device)

    from sdmi.trainer import DDPMTrainer, S_LOSS, S_NORM, S_SKIP
    from sdmi import kernels as K
    import models.unet_cond_base as mc

    wl = WORKLOADS[args.workload]
    is_dit = args.workload == "dit"
    is_uncond = args.workload == "uncond-unet"
    if args.workload == "vqvae":
        return main_vqvae(args, wl, world, rank, device)
    if args.workload == "sample":
        return main_sample(args, wl, world, rank, device)
    if args.workload == "vqvae-train":
        return main_vqvae_train(args, wl, world, rank, device)
    cfg = dit_config() if is_dit else (uncond_config() if is_uncond else cond_config())
    torch.manual_seed(1111)  # identical initial weights on every rank (DDP broadcasts rank 0's)
    group = dist.group.WORLD if (world > 1 or forced) else None
    red_kw = dict(force_reducer=True) if forced else {}
    single = args.issue == "graph" and world == 1  # single-stream hipGraph capture (weight gradients inline)
    if is_dit:
        from models.transformer import DIT
        init = DIT(4, cfg).state_dict()
        for k, v in init.items():  # the reference zero-initialises adaLN / proj_out: give them random values so
            if v.abs().max() == 0:  # the timed step runs on non-trivial data (zeros clock higher, MI355X DVFS)
                v.normal_(0.0, 0.02)
        trainer = DDPMTrainer(cfg, init, device, base="dit", lr=1e-4, ema_decay=None, group=group,
                              grad_wire=args.grad_wire, single_stream=single, **red_kw)
    elif is_uncond:  # tools/train_ddpm_vqvae.py:76-104: Adam(ldm_lr 5e-6, celebhq.yaml:54), no clip, no EMA
        import models.unet_base as mu
        init = mu.Unet(4, cfg).state_dict()
        trainer = DDPMTrainer(cfg, init, device, base="uncond", lr=5e-6, ema_decay=None, max_grad_norm=float("inf"),
                              sched=(1000, 0.0015, 0.0195), group=group, grad_wire=args.grad_wire,
                              single_stream=single, **red_kw)
    else:
        init = mc.Unet(4, cfg).state_dict()
        trainer = DDPMTrainer(cfg, init, device, group=group, grad_wire=args.grad_wire, single_stream=single, **red_kw)
    B = args.batch
    x0, text, empty, mask = synthetic_batch(B, device, 1111 + rank)
    gen = torch.Generator(device=device).manual_seed(1111 + rank)

    drop_p = 0.9 if is_dit else 0.1  # image cond-drop (Model_DiT_12L_config: 0.9; celebhq_text_image_cond: 0.1)

    def eager_step():
        noise = torch.randn(x0.shape, device=device, generator=gen)
        t = torch.randint(0, 1000, (B,), device=device, generator=gen)
        if is_uncond:
            trainer.step(x0, noise, t)
            return
        if is_dit:  # image-only conditioning, drop prob 0.9 (Model_DiT_12L_config.py ldm_image_condition_cond_drop_prob)
            keep = (torch.rand(B, device=device, generator=gen) > 0.9).float()
            trainer.step(x0, noise, t, None, mask, mask_keep=keep)
            return
        drop_t = torch.rand(B, device=device, generator=gen) < 0.1       # diffusion_utils.py:21-28
        txt = torch.where(drop_t[:, None, None], empty, text)
        keep = (torch.rand(B, device=device, generator=gen) > 0.1).float()  # diffusion_utils.py:31-37
        trainer.step(x0, noise, t, txt, mask, mask_keep=keep)

    issue = args.issue
    if issue == "graph" and world > 1:
        issue = "plan"
    if issue != "eager":
        from sdmi.graph import CapturedTrainStep
        cap = CapturedTrainStep(trainer, x0, None if (is_dit or is_uncond) else text, empty, None if is_uncond else mask,
                                B, generator=gen, drop_p=drop_p,
                                mode=issue)
        one_step = cap.step
    else:
        one_step = eager_step

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = e.item()
    steps_per_s = args.steps / elapsed
    state = trainer.state.tolist()

    # dominant-kernel roofline: the implicit-GEMM conv/linear launches of PROF_STEPS extra (untimed) steps, timed
    # with HIP events on the stream they run on (averaged over the steps: one step's concurrency noise is ~10 %)
    roof = None
    if args.profile_gemm:
        PROF_STEPS = 3
        K.PROFILE = []
        tails = []
        if trainer.reducer is not None:
            trainer.measure_exchange_tail()
        for _ in range(PROF_STEPS):
            eager_step()
            if trainer.reducer is not None:
                torch.cuda.synchronize()
                tails.append(trainer.exchange_tail_ms())
        trainer.measure_exchange_tail(False)
        torch.cuda.synchronize()
        prof, K.PROFILE = K.PROFILE, None
        roof = gemm_roofline(prof, PROF_STEPS, args.workload)

    FLOP = wl["flop"]
    result = {
        "metric": wl["metric"], "value": steps_per_s * world, "unit": "steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1000.0 / steps_per_s, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic (seeded CelebHQ-shaped latents, text, masks; "
                                                        "random-init weights of the reference architecture)",
        "config": ({"workload": "DiT-12L Model_DiT_12L_config training step (image cond, no EMA, lr 1e-4)",
                    "model": "DiT-12L 18.3M", "global_batch": B * world, "per_gpu_batch": B, "latent": [4, 32, 32],
                    "mask": [18, 512, 512], "parallelism": f"dp{world}"} if is_dit else
                   {"workload": "uncond-UNet celebhq.yaml training step (Adam lr 5e-6, no clip / EMA)",
                    "model": "uncond-UNet 103.5M", "global_batch": B * world, "per_gpu_batch": B,
                    "latent": [4, 32, 32], "parallelism": f"dp{world}"} if is_uncond else
                   {"workload": "cond-UNet celebhq_text_image_cond training step", "model": "cond-UNet 118.5M",
                    "global_batch": B * world, "per_gpu_batch": B, "latent": [4, 32, 32],
                    "text": [77, 512], "mask": [18, 512, 512], "parallelism": f"dp{world}"}),
        "per_gpu_steps_per_s": steps_per_s, "samples_per_s": steps_per_s * B * world,
        "model_flops_utilization": FLOP * steps_per_s / PEAK_BF16,
        "last_loss": state[S_LOSS], "last_grad_norm": state[S_NORM], "last_step_skipped": bool(state[S_SKIP]),
        "issue": issue,
        "roofline": roof,
    }
    if forced:
        result["forced_reducer"] = {
            "note": "N = 1 with the N > 1 gradient path on: RCCL group of one rank, bucketed all-reduce on the reducer "
                    "stream (identities at one rank), per-bucket norm blocks; compare ms_per_step with the plain line",
            "backend": dist.get_backend(), "bucket_bytes": trainer.reducer.bucket * trainer.store.grads.element_size(),
            "issue": ("library RCCL communicator, native plan ops (csrc/comm.hip)" if trainer.reducer.comm is not None
                      else "torch.distributed callouts")}
        result["config"]["parallelism"] = "dp1 + forced reducer"
    if world > 1 or forced:
        result["collectives"] = collectives
        result["grad_wire"] = trainer.grad_wire
        if args.profile_gemm and tails:
            # exposed gradient exchange: compute-stream time from the end of the backward (all gradients final) to the
            # last bucket's all-reduce waited for, eager profiled steps (HIP events), max over ranks
            tail = torch.tensor([sum(tails) / len(tails)], device=device, dtype=torch.float64)
            dist.all_reduce(tail, op=dist.ReduceOp.MAX)
            result["exchange_tail_ms"] = tail.item()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_dit(cfg) if is_dit else cpu_baseline(cfg, uncond=is_uncond)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1 or forced:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
