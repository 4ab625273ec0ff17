from .checkpoint import load_checkpoint, load_model_state_for_export, read_meta, save_checkpoint
from .hf import load_hf_weights, load_safetensors_state_dict, save_hf_folder

__all__ = ["load_checkpoint", "load_model_state_for_export", "read_meta", "save_checkpoint", "load_hf_weights",
           "load_safetensors_state_dict", "save_hf_folder"]
