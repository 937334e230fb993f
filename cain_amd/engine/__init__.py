"""Decode engine (on-device arm)."""
from .engine import OLLAMA_DEFAULTS, DecodeEngine, GenResult  # noqa: F401
