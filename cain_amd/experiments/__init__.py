"""The reference study as native RunnerConfigs (``study.StudyConfig``); thin per-config files live in the
repository's ``experiments/`` directory."""
from .study import StudyConfig, StudySettings, load_topics, prompt_for

__all__ = ["StudyConfig", "StudySettings", "load_topics", "prompt_for"]
