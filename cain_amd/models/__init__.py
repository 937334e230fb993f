"""Model zoo: the study's seven architectures, random-init weights, real checkpoints (Hugging Face directories, GGUF
files, a local Ollama store), torch-eager oracle."""
from .config import MODELS, STUDY_ORDER, TINY, ModelConfig, get_config  # noqa: F401
from .gguf import export_gguf, load_gguf  # noqa: F401
from .hf import load_pretrained, ollama_blob, registered_checkpoints  # noqa: F401
from .weights import ModelWeights, pack_for_engine, random_weights  # noqa: F401
