"""Observability and misc helpers."""
from .obs import MetricsWriter, PhaseTimer, Telemetry

__all__ = ["MetricsWriter", "PhaseTimer", "Telemetry"]
