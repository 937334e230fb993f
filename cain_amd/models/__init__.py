"""Model zoo: the study's seven architectures, random-init weights, torch-eager oracle."""
from .config import MODELS, STUDY_ORDER, TINY, ModelConfig, get_config  # noqa: F401
from .weights import ModelWeights, pack_for_engine, random_weights  # noqa: F401
