"""cain_amd — MI355X-native on-device vs remote LLM energy benchmarking framework.

Subpackages
-----------
runner    reference-compatible experiment orchestration (RunnerConfig hooks, run table, resume, CLI)
energy    native amd-smi energy sampler + profiler plugin (replaces codecarbon/powermetrics)
models    the 7 architectures of the study, random-init weights, torch-eager oracle
ops       hand-written HIP/CDNA4 kernels (gfx950) + bindings
engine    autoregressive decode engine (KV cache, HIP-graph decode step, sampling)
serve     Ollama-compatible HTTP server over the engine
client    Ollama-compatible HTTP client (captures token counts)
parallel  one-process-per-GPU data-parallel trial fan-out over RCCL
analysis  statistics of the paper's notebook (IQR filter, Wilcoxon, Cliff's delta, Spearman)
utils     shared helpers
"""
__version__ = "0.1.0"
