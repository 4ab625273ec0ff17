from .base import BaseModel, BaseModelConfig, CausalLMOutput
from .llama import Llama, LlamaConfig

__all__ = ["BaseModel", "BaseModelConfig", "CausalLMOutput", "Llama", "LlamaConfig"]


def __getattr__(name):
    if name in ("Phi3", "Phi3Config"):
        from . import phi3
        return getattr(phi3, name)
    if name in ("HFCausalLM", "HFCausalLMConfig"):
        from . import hf_causal_lm
        return getattr(hf_causal_lm, name)
    raise AttributeError(name)
