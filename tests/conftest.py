import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "stablediffusion-pytorch_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    if os.environ.get("SDMI_LIB_PATH"):
        # the override exists for A/B timing scripts; parity results must come from the in-tree build
        raise pytest.UsageError(f"SDMI_LIB_PATH={os.environ['SDMI_LIB_PATH']} is set: the tests run only against the "
                                "in-tree libsdmi.so (unset it)")
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libsdmi.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


# Tests that pin the five BASELINE configs and the training-step failure semantics (a19) run first, so that with `-x`
# a later failure cannot hide them from a driver run (config 1 MNIST LDM, config 2 VQVAE CelebHQ-256, config 3 uncond
# UNet, config 4 cond UNet + the B=32 headline step, config 5 DiT-12L, then GradScaler / non-finite-rank semantics).
PRIORITY = (
    "test_mnist_gpu.py::test_mnist_unet_forward_backward",
    "test_mnist_gpu.py::test_mnist_trainer_two_steps",
    "test_vqvae_gpu.py::test_encode_decode_vs_reference[vqvae_celebhq256",
    "test_unet_gpu.py::test_full_unet_forward_backward_b2[False]",
    "test_unet_gpu.py::test_full_unet_forward_backward_b2[True]",
    "test_unet_gpu.py::test_full_cond_forward_matches_golden",
    "test_bench_step_gpu.py::test_bench_step_b32_plan_replay_matches_oracle",
    "test_dit_gpu.py::test_dit12l_forward_backward_b2",
    "test_dit_gpu.py::test_dit12l_forward_matches_golden",
    "test_gradscaler_gpu.py::",
    "test_dp_gpu.py::test_two_rank_nonfinite_loss_on_one_rank_skips_everywhere",
    "test_sampling_gpu.py::test_captured_ddim_matches_stepwise",
)


def _priority(item):
    nid = item.nodeid.split("/")[-1]
    for i, p in enumerate(PRIORITY):
        if nid.startswith(p):
            return i
    return len(PRIORITY)


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        items.sort(key=_priority)  # stable: everything else keeps its file order
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _device_sync_after_gpu_test(request):
    """Drain every stream after each GPU test, so an asynchronous device fault is reported by the test whose kernels
    caused it (not by whichever later test next touches the device)."""
    yield
    if "gpu" in request.keywords:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
