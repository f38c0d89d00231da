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
    config.addinivalue_line("markers", "miopen_ref: DenseNet/VGG-only eager reference, which runs on MIOpen "
                                       "(guard-page clean, profiles/fault_attribution_r6.md)")


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


@pytest.fixture(autouse=True)
def _miopen_reference(request):
    """Tests marked ``miopen_ref`` build eager references of DenseNet/VGG only, whose MIOpen
    convolutions ran clean under the guard-page allocator (tools/guard_pages.py): they use MIOpen,
    which is several times faster than PyTorch's native fp32 convolutions at batch 256.  MobileNetV2
    references stay on the native convolutions."""
    if request.node.get_closest_marker("miopen_ref") is None or os.environ.get("IDC_EAGER_MIOPEN") == "0":
        yield
        return
    prev = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = True
    try:
        yield
    finally:
        torch.backends.cudnn.enabled = prev
