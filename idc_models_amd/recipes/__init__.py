from .federated import FedConfig, SecureConfig, run_fedavg, run_secure
from .transfer import PRESETS, TransferConfig, run_transfer_learning

__all__ = ["FedConfig", "SecureConfig", "run_fedavg", "run_secure", "PRESETS", "TransferConfig",
           "run_transfer_learning"]
