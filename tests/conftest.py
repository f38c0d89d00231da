import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    # Eager-PyTorch reference runs use PyTorch's native convolutions, not MIOpen: a MIOpen kernel
    # of the eager MobileNetV2 batch-32 backward accesses memory past the end of a tensor.  It
    # faults deterministically with no fused program in the process once every tensor ends at an
    # unmapped page (tools/guard_pages.py), and in the suite whenever earlier tests leave a tensor
    # at a segment end (profiles/fault_attribution_r6.md).  IDC_EAGER_MIOPEN=1 selects MIOpen.
    if os.environ.get("IDC_EAGER_MIOPEN", "0") != "1":
        torch.backends.cudnn.enabled = False
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)
    yield
