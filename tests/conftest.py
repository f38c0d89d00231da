import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    # Eager-PyTorch REFERENCE runs use PyTorch's native convolutions, not MIOpen: since round 5 a
    # MIOpen kernel faults the GPU inside an eager MobileNetV2 backward when earlier eager runs are in
    # the same process (the round-4 tree faults the same way on the same boxes).  Our fused path never
    # calls MIOpen; the variable reaches the worker subprocesses too (idc_models_amd/__init__.py).
    os.environ.setdefault("IDC_EAGER_MIOPEN", "0")
    if os.environ["IDC_EAGER_MIOPEN"] == "0":
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
