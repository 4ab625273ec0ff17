from .base import BaseDataModule, BaseDataModuleConfig, ResumableDistributedSampler
from .dummy import DummyDataModule, DummyDataModuleConfig
from .hf_based import HFBasedDataModule, HFBasedDataModuleConfig
from .instruction_tuning import (InstructionTuningDataCollator, InstructionTuningDataModule,
                                 InstructionTuningDataModuleConfig)
from .preference_tuning import (PreferenceTuningDataCollator, PreferenceTuningDataModule,
                                PreferenceTuningDataModuleConfig)
from .pre_training import PreTrainingDataCollator, PreTrainingDataModule, PreTrainingDataModuleConfig

__all__ = ["BaseDataModule", "BaseDataModuleConfig", "ResumableDistributedSampler", "DummyDataModule",
           "DummyDataModuleConfig", "HFBasedDataModule", "HFBasedDataModuleConfig", "InstructionTuningDataCollator",
           "InstructionTuningDataModule", "InstructionTuningDataModuleConfig", "PreferenceTuningDataCollator",
           "PreferenceTuningDataModule", "PreferenceTuningDataModuleConfig", "PreTrainingDataCollator",
           "PreTrainingDataModule", "PreTrainingDataModuleConfig"]
