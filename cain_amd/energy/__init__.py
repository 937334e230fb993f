"""Energy / utilisation measurement (replaces codecarbon + powermetrics + psutil loop)."""
from .meter import EnergyMeter, EnergyReading, resolve_smi_indices  # noqa: F401
from .plugin import DataColumns, emission_tracker  # noqa: F401
