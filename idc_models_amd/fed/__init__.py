"""Federated learning: FedAvg (TFF semantics) and secure aggregation, simulated over one node."""
from .fedavg import (FedAvgProcess, FederatedEvaluation, ModelWeights, ServerState, assign_clients,
                     broadcast_server_state, build_federated_averaging_process, build_federated_evaluation,
                     load_server_extra, load_server_state, save_server_state, state_with_new_model_weights)
from .secure import SecureFederatedProcess

__all__ = ["FedAvgProcess", "FederatedEvaluation", "ModelWeights", "ServerState", "assign_clients",
           "broadcast_server_state", "build_federated_averaging_process", "build_federated_evaluation",
           "load_server_extra", "load_server_state", "save_server_state", "state_with_new_model_weights",
           "SecureFederatedProcess"]
