"""Trust layer: graph analytics, anomaly filters, blockchain ledger, reference network fixture."""
from . import graph, netdata
from .anomaly import UpdateAnomalyFilter, Verdicts, topology_filter
from .ledger import Ledger, block_hash, block_preimage

__all__ = ["graph", "netdata", "UpdateAnomalyFilter", "Verdicts", "topology_filter", "Ledger",
           "block_hash", "block_preimage"]
