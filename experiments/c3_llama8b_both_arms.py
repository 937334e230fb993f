"""Config 3 — llama3.1:8b on-device vs remote at the three output lengths on 1x MI355X (the paper's
headline comparison for its largest model).  Remote: SERVER_IP from .env, else a modelled remote server.

    python -m cain_amd experiments/c3_llama8b_both_arms.py
"""
from cain_amd.experiments import StudyConfig, StudySettings


class RunnerConfig(StudyConfig):
    SETTINGS = StudySettings(name="c3_llama8b_both_arms", models=["llama3.1:8b"], repetitions=30,
                             cooldown_ms=5000)
