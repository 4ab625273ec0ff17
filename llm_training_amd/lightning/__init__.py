"""Compatibility namespace: reference YAML names ``llm_training.lightning.<X>`` resolve here
(src/llm_training/lightning/__init__.py exports strategies, callbacks and the W&B logger)."""
from ..runtime.callbacks import (ExtraConfig, LearningRateMonitor, ModelCheckpoint, OutputRedirection,
                                 SaveConfigCallback, TQDMProgressBar, TrainingTimeEstimator)
from ..runtime.loggers import CSVLogger, JSONLLogger, WandbLogger
from ..runtime.strategies import DDPStrategy, DeepSpeedStrategy, FSDP2Strategy, SingleDeviceStrategy
from ..runtime.trainer import Trainer

__all__ = ["ExtraConfig", "LearningRateMonitor", "ModelCheckpoint", "OutputRedirection", "SaveConfigCallback",
           "TQDMProgressBar", "TrainingTimeEstimator", "CSVLogger", "JSONLLogger", "WandbLogger", "DDPStrategy",
           "DeepSpeedStrategy", "FSDP2Strategy", "SingleDeviceStrategy", "Trainer"]
