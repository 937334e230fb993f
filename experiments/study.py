"""Config 5 — the full factorial study: 7 models x {remote, on_device} x {100, 500, 1000} words x 30
repetitions (1,260 runs, reference experiment/RunnerConfig.py:66-87), trials fanned out data-parallel:

    python -m cain_amd experiments/study.py --gpus 8

Every rank starts its own on-device server on its GPU; the remote arm talks to ``SERVER_IP`` from ``.env``
(or a modelled server when unset; ``CAIN_STUDY_REMOTE=local:<gpu>`` serves it from one engine server on that GPU
of the node, started once by rank 0 and shared by every rank).
"""
from cain_amd.experiments import StudyConfig, StudySettings


class RunnerConfig(StudyConfig):
    SETTINGS = StudySettings(name="full_factorial", cooldown_ms=10000, max_batch=4)
