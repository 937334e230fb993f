"""Config 1 — qwen2:1.5b, remote-HTTP arm only, CPU orchestrator, no GPU: exercises the runner, the HTTP
client, the Ollama-compatible server (the real qwen2:1.5b architecture on the CPU engine backend, random
weights) and run_table.csv output end to end.

    python -m cain_amd experiments/c1_remote_qwen2_cpu.py
"""
from cain_amd.experiments import StudyConfig, StudySettings


class RunnerConfig(StudyConfig):
    SETTINGS = StudySettings(name="c1_remote_qwen2_cpu", models=["qwen2:1.5b"], methods=["remote"],
                             lengths=["100"], repetitions=3, cooldown_ms=0, remote="local:cpu", max_batch=1)
