"""Distributed runtime: process groups, flat buffers, FedAvg all-reduce, P2P gossip."""
from .dist import (Runtime, init_runtime, runtime, shutdown, barrier, all_reduce_, broadcast_,
                   all_gather_tensor, all_gather_object, max_over_ranks, p2p_exchange, P2PHandle)
from .flat import FlatParams, FlatAdamW
from .topology import neighbours, mixing_matrix, client_rank, clients_of_rank
from .gossip import GossipEngine

__all__ = ["Runtime", "init_runtime", "runtime", "shutdown", "barrier", "all_reduce_", "broadcast_",
           "all_gather_tensor", "all_gather_object", "max_over_ranks", "p2p_exchange", "P2PHandle",
           "FlatParams", "FlatAdamW", "neighbours", "mixing_matrix", "client_rank",
           "clients_of_rank", "GossipEngine"]
