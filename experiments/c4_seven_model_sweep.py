"""Config 4 — the 7-model on-device sweep (gemma:2b/7b, phi3:3.8b, qwen2:1.5b/7b, mistral:7b, llama3.1:8b)
on 1x MI355X; all seven models stay resident in HBM (~80 GB of bf16 weights of 288 GB).

    python -m cain_amd experiments/c4_seven_model_sweep.py
"""
from cain_amd.experiments import StudyConfig, StudySettings


class RunnerConfig(StudyConfig):
    SETTINGS = StudySettings(name="c4_seven_model_sweep", methods=["on_device"], repetitions=30, cooldown_ms=5000)
