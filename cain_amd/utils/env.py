"""``.env`` loading (python-dotenv is not installed in this image).

The reference reads ``SERVER_IP`` from a git-ignored ``.env`` in the repo root
(README.md:25-28, experiment/RunnerConfig.py:125-126), with lines of the form
``export SERVER_IP=...``.  ``load_dotenv`` accepts ``KEY=VAL``, ``export KEY=VAL``,
quotes and comments, and never overrides variables already set in the
environment (python-dotenv's default).
"""
from __future__ import annotations

import os
import shlex
from pathlib import Path
from typing import Dict, Optional, Union


def dotenv_values(path: Union[str, Path] = ".env") -> Dict[str, str]:
    p = Path(path)
    out: Dict[str, str] = {}
    if not p.is_file():
        return out
    for raw in p.read_text().splitlines():
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        if line.startswith("export "):
            line = line[len("export "):].strip()
        if "=" not in line:
            continue
        k, v = line.split("=", 1)
        k = k.strip()
        v = v.strip()
        if v and v[0] in "\"'":
            try:
                v = shlex.split(v)[0]
            except ValueError:
                v = v.strip("\"'")
        else:
            v = v.split(" #", 1)[0].strip()
        out[k] = v
    return out


def load_dotenv(path: Union[str, Path, None] = None, override: bool = False) -> bool:
    candidates = [Path(path)] if path else [Path.cwd() / ".env"]
    found = False
    for p in candidates:
        vals = dotenv_values(p)
        if vals:
            found = True
        for k, v in vals.items():
            if override or k not in os.environ:
                os.environ[k] = v
    return found


def server_url(method: str, env_var: str = "SERVER_IP", port: int = 11434, local: str = "127.0.0.1") -> str:
    """URL of the Ollama-compatible endpoint for an arm: localhost for on_device, ``$SERVER_IP`` otherwise
    (reference experiment/RunnerConfig.py:122-126).  ``SERVER_IP`` may carry a port (``host:port``)."""
    if method == "on_device":
        host = os.environ.get("CAIN_LOCAL_SERVER", f"{local}:{port}")
    else:
        load_dotenv()
        host = os.environ.get(env_var)
        if not host:
            raise RuntimeError(f"{env_var} is not set (put `export {env_var}=<host>` in .env)")
    if ":" not in host.split("//")[-1]:
        host = f"{host}:{port}"
    return host if "://" in host else f"http://{host}"
