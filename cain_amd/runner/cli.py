"""Command-line entry point: ``python -m cain_amd <config.py | command> [options]``.

Reference: experiment-runner/__main__.py:17-79 and ConfigValidator/
CLIRegister/CLIRegister.py:14-125.  ``python -m cain_amd path/to/RunnerConfig.py``
loads the file, instantiates ``RunnerConfig``, fingerprints the source,
validates, and runs the experiment; any other first argument is a command.

Commands: ``help``, ``config-create [dir]``, ``prepare`` (build the native
libraries and HIP kernels in-tree), ``analyze <run_table.csv>`` (paper tables),
``serve`` (Ollama-compatible server on this host's GPU), ``generate``
(one local generation, prints Ollama-style JSON).

Run options (new): ``--gpus N`` fans TODO rows out data-parallel over N GPU
worker processes (``cain_amd.parallel``; ``--max-restarts`` relaunches after a
rank dies, ``--retry-failed`` re-runs failed rows), ``--isolation``, ``--timeout``,
``--cooldown-ms``, ``--yes`` (answer the md5 prompt), ``--seed``,
``--dry-run`` (validate and print the run table only).
"""
from __future__ import annotations

import argparse
import importlib.util
import os
import shutil
import sys
import traceback
import uuid
from pathlib import Path
from typing import List, Optional

from tabulate import tabulate

from .errors import BaseError, CommandNotRecognisedError, ConfigInvalidClassNameError, InvalidUserSpecifiedPathError
from .output import BashHeaders, OutputProcedure as output
from .paths import is_path_exists_or_creatable


def load_config_module(path: str):
    from . import compat

    compat.install()
    path = os.path.abspath(path)
    name = Path(path).stem
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def build_config(path: str):
    from .fingerprint import fingerprint

    mod = load_config_module(path)
    if not hasattr(mod, "RunnerConfig"):
        raise ConfigInvalidClassNameError()
    config = mod.RunnerConfig()
    source = Path(path).read_text()
    return config, fingerprint(source, path), source


# ---------------------------------------------------------------------- commands
def cmd_help(_args=None) -> None:
    print(BashHeaders.BOLD + "--- EXPERIMENT_RUNNER HELP ---" + BashHeaders.ENDC)
    print("\n%-*s  %s" % (10, "Usage:", "python -m cain_amd <path_to_config.py> [--gpus N] [--yes] ..."))
    print("%-*s  %s" % (10, "Utility:", "python -m cain_amd <command>"))
    print("\nAvailable commands:\n")
    print(tabulate([(k, v[0]) for k, v in COMMANDS.items()], ["Command", "Parameters"]))
    print("\nHelp can be called for each command:")
    print(BashHeaders.WARNING + "example: " + BashHeaders.ENDC + "python -m cain_amd prepare help")


def cmd_config_create(args: List[str]) -> None:
    from . import template

    dest = Path(args[0]) if args else Path.cwd() / "experiments"
    if not is_path_exists_or_creatable(str(dest)):
        raise InvalidUserSpecifiedPathError(dest)
    dest.mkdir(parents=True, exist_ok=True)
    name = f"RunnerConfig-{uuid.uuid1()}.py"
    shutil.copyfile(template.__file__, dest / name)
    output.console_log_OK(f"Successfully created new config with unique identifier in: {dest}\n"
                          f"With the unique name (please rename): {name}")


def cmd_prepare(args: List[str]) -> None:
    from .. import build

    build.build_all(verbose=True)


def cmd_analyze(args: List[str]) -> None:
    from ..analysis import report

    report.main(args)


def cmd_serve(args: List[str]) -> None:
    from ..serve import server

    server.main(args)


def cmd_generate(args: List[str]) -> None:
    from ..serve import server

    server.generate_main(args)


def cmd_convert(args: List[str]) -> None:
    """``convert <checkpoint dir | .gguf> <out.gguf> [--type F16]``: a checkpoint as a GGUF file with llama.cpp's
    conventions (models/gguf.py export_gguf), e.g. to run the same weights under llama.cpp / Ollama.  A Hugging Face
    directory's byte-level or SentencePiece-style BPE ``tokenizer.json`` and chat template go into the file's
    ``tokenizer.ggml.*`` metadata (gguf_tokenizer_fields) and its context length is the checkpoint's
    ``max_position_embeddings``; a vocabulary with no GGUF form (e.g. word-level) is left out, and the file then loads
    only where a tokenizer is supplied separately (this package's engine with token ids)."""
    import json

    import torch

    from ..models.gguf import ARCHS, GGUFFile, export_gguf, gguf_tokenizer_fields, is_gguf
    from ..models.hf import _chat_template, load_pretrained

    ap = argparse.ArgumentParser(prog="python -m cain_amd convert")
    ap.add_argument("src", help="a Hugging Face checkpoint directory or a GGUF file")
    ap.add_argument("dst", help="the GGUF file to write")
    ap.add_argument("--type", default="F16", choices=["F32", "F16", "BF16", "Q8_0", "Q4_0"])
    ap.add_argument("--arch", default=None, choices=list(ARCHS),
                    help="GGUF architecture (default: from the checkpoint; Mistral is written as llama)")
    ns = ap.parse_args(args)
    cfg, mw, _ = load_pretrained(ns.src, dtype=torch.float32)
    arch = ns.arch
    if arch is None:
        arch = {"mistral": "llama"}.get(cfg.family, cfg.family)
        if arch not in ARCHS:
            raise SystemExit(f"cannot tell the GGUF architecture of {ns.src}: pass --arch")
        print(f"architecture: {arch} (pass --arch to override)")
    src = Path(ns.src)
    fields, ctx = None, None
    if is_gguf(src):
        md = GGUFFile(src).metadata  # a GGUF source keeps its own vocabulary and context length
        fields = {k: v for k, v in md.items() if k.startswith("tokenizer.")}
        ctx = md.get(f"{md.get('general.architecture')}.context_length")
    else:
        conf = json.loads((src / "config.json").read_text())
        ctx = conf.get("max_position_embeddings")
        if (src / "tokenizer.json").exists():
            fields = gguf_tokenizer_fields(json.loads((src / "tokenizer.json").read_text()), cfg.bos_id, cfg.eos_id,
                                           _chat_template(src)[0])
            if fields is None:
                print("tokenizer.json is not a BPE vocabulary GGUF can hold: written without tokenizer metadata")
    export_gguf(mw, ns.dst, arch, tensor_type=ns.type, tokenizer_fields=fields, context_length=ctx)
    print(f"wrote {ns.dst}: {cfg.n_layers} layers, d {cfg.d_model}, {ns.type}"
          f"{', tokenizer ' + fields['tokenizer.ggml.model'] if fields else ''}")


COMMANDS = {
    "config-create": ("[path_to_user_specified_dir]", cmd_config_create),
    "prepare": ("", cmd_prepare),
    "analyze": ("<run_table.csv> [--out DIR]", cmd_analyze),
    "serve": ("[--host H] [--port P] [--models m1,m2] [--device N]", cmd_serve),
    "generate": ("--model M --prompt P [--num-predict N] [--checkpoint PATH]", cmd_generate),
    "convert": ("<checkpoint dir | .gguf> <out.gguf> [--type F16|Q8_0|Q4_0|...]", cmd_convert),
    "help": ("", cmd_help),
}


def run_experiment(argv: List[str]) -> None:
    ap = argparse.ArgumentParser(prog="python -m cain_amd <config.py>")
    ap.add_argument("config")
    ap.add_argument("--gpus", type=int, default=0, help="data-parallel GPU workers (0 = run in this process)")
    ap.add_argument("--isolation", choices=["fork", "inline", "spawn"], default=None)
    ap.add_argument("--timeout", type=float, default=None, help="per-run wall-clock limit (s)")
    ap.add_argument("--cooldown-ms", type=int, default=None)
    ap.add_argument("--yes", action="store_true", help="continue on md5 mismatch without asking")
    ap.add_argument("--seed", type=int, default=None, help="seed for the run-table shuffle")
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--max-restarts", type=int, default=0,
                    help="with --gpus: relaunch after a rank dies, resuming the TODO rows (elastic restart)")
    ap.add_argument("--retry-failed", type=int, default=0, help="with --gpus: extra passes over failed runs")
    ns = ap.parse_args(argv)
    if ns.cooldown_ms is not None:
        os.environ["CAIN_COOLDOWN_MS"] = str(ns.cooldown_ms)
    if ns.seed is not None:
        os.environ["CAIN_SHUFFLE_SEED"] = str(ns.seed)
    if ns.gpus and ns.gpus > 0:
        from ..parallel.fanout import launch

        sys.exit(launch(ns.config, ns.gpus, isolation=ns.isolation, timeout=ns.timeout,
                        assume_yes=True if ns.yes else None, retry_failed=ns.retry_failed,
                        max_restarts=ns.max_restarts))
    from .controller import ExperimentController
    from .validator import ConfigValidator

    config, metadata, source = build_config(ns.config)
    ConfigValidator.validate_config(config)
    if ns.dry_run:
        table = config.create_run_table_model().generate_experiment_run_table()
        print(tabulate([[r[k] for k in list(r)[:6]] for r in table[:50]], list(table[0])[:6]))
        output.console_log_OK(f"dry run: {len(table)} runs")
        return
    ExperimentController(config, metadata, source=source, source_name=ns.config,
                         assume_yes=True if ns.yes else None, isolation=ns.isolation,
                         run_timeout_s=ns.timeout).do_experiment()


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    try:
        if not argv:
            cmd_help()
        elif argv[0].endswith(".py"):
            run_experiment(argv)
        else:
            entry = COMMANDS.get(argv[0])
            if entry is None:
                raise CommandNotRecognisedError(argv[0])
            if len(argv) > 1 and argv[1] == "help":
                print(f"{argv[0]} {entry[0]}\n\n{(entry[1].__doc__ or '').strip()}")
            else:
                entry[1](argv[1:])
        return 0
    except BaseError as e:
        print(f"\n{e}")
        return 1
    except SystemExit:
        raise
    except Exception:
        traceback.print_exc()
        return 1
