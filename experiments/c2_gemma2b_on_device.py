"""Config 2 — gemma:2b on-device decode (bf16, HIP kernels) on 1x MI355X with amd-smi energy sampling.

    python -m cain_amd experiments/c2_gemma2b_on_device.py
"""
from cain_amd.experiments import StudyConfig, StudySettings


class RunnerConfig(StudyConfig):
    SETTINGS = StudySettings(name="c2_gemma2b_on_device", models=["gemma:2b"], methods=["on_device"],
                             repetitions=30, cooldown_ms=5000)
