"""idc_models_amd: MI355X-native training framework for the IDC classification models.

``IDC_EAGER_MIOPEN=0`` makes the eager (plain torch.nn) backend use PyTorch's native convolutions
instead of MIOpen; the fused backend's HIP kernels never call MIOpen.  The GPU test suite sets it
for its eager reference runs (tests/conftest.py).
"""
import os as _os

if _os.environ.get("IDC_EAGER_MIOPEN", "1") == "0":
    import torch as _torch

    _torch.backends.cudnn.enabled = False
