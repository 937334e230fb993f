"""Ollama-compatible HTTP clients (in-process and curl), capturing token counts."""
from .ollama import CurlRequest, GenerateResponse, OllamaClient, OllamaError  # noqa: F401
