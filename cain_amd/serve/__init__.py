"""Ollama-compatible server over the decode engine."""
from .server import (Backend, EngineBackend, FakeBackend, ServerThread, default_num_predict,  # noqa: F401
                     make_server)
