"""bench.py's host logic on the CPU: which kernel instantiation a profiled GEMM launch is (the roofline's kernel
glob), and which committed PMC evidence the roofline line quotes -- the newest file for the workload, reported as
measured on the running tree exactly when its source digest is the tree's (sdmi._build.source_digest)."""
import glob
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_kernel_glob_matches_its_instantiations_only():
    k2 = bench.kernel_name("gemm_a2b2", "variant=2 tile_n=128 bytes=1")
    assert k2 == "gemm_dma_kernel<2, 2, 2, 128, 128, 2, *, 64, *, 1>"
    name = ("void (anonymous namespace)::gemm_dma_kernel<2, 2, 2, 128, 128, 2, 1, 64, false, 1>"
            "((anonymous namespace)::Args, (anonymous namespace)::EpiArgs)")
    assert bench.kernel_matches(k2, name)  # the RED = 1 instantiation belongs to the same kernel
    assert not bench.kernel_matches(bench.kernel_name("gemm_a2b2", "variant=11 tile_n=128"), name)  # k-groups
    assert not bench.kernel_matches(bench.kernel_name("gemm_a1b0", "variant=2 tile_n=128"), name)   # other modes
    assert bench.kernel_name("gemm_a0b0", "variant=0 tile_n=128") == "gemm_kernel<0, 0, *>"


@pytest.mark.parametrize("workload", ["cond-unet", "dit", "uncond-unet"])
def test_roofline_evidence_is_the_newest_and_digest_tagged(workload):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "stablediffusion-pytorch_amd"))
    from sdmi import _build
    w = workload.replace("-", "_")
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{w}_roofline_evidence.json")))
    if not files:
        pytest.skip(f"no committed roofline evidence for {workload}")
    ev = json.load(open(files[-1]))
    traffic, src = bench.pmc_traffic(workload, ev["kernel"], ev["launches"] == "unsplit")  # the set the bench timed
    assert traffic is not None and traffic > 0
    assert src["file"] == os.path.basename(files[-1])
    assert src["measured_on_this_tree"] == (src["tree_digest"] == _build.source_digest())
