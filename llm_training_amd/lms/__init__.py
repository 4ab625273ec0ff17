from .base import BaseLM, BaseLMConfig, BaseOptimizerConfig, ModelProvider
from .clm import CLM, CLMConfig
from .preference import DPO, ORPO, DPOConfig, ORPOConfig

__all__ = ["BaseLM", "BaseLMConfig", "BaseOptimizerConfig", "ModelProvider", "CLM", "CLMConfig", "DPO", "DPOConfig",
           "ORPO", "ORPOConfig"]
