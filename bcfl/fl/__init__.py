"""Federated learning layer: clients, server FedAvg, serverless gossip, virtual clients."""
from .client import Client
from .federation import Federation, weighted_average
from .trainer import EvalResult, LocalTrainer

__all__ = ["Client", "Federation", "weighted_average", "EvalResult", "LocalTrainer"]
