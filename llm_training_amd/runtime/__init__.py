from .callbacks import (ExtraConfig, LearningRateMonitor, ModelCheckpoint, OutputRedirection, SaveConfigCallback,
                        TQDMProgressBar, TrainingTimeEstimator)
from .loggers import CSVLogger, JSONLLogger, WandbLogger
from .strategies import DDPStrategy, DeepSpeedStrategy, FSDP2Strategy, SingleDeviceStrategy, Strategy
from .trainer import Trainer

__all__ = ["ExtraConfig", "LearningRateMonitor", "ModelCheckpoint", "OutputRedirection", "SaveConfigCallback",
           "TQDMProgressBar", "TrainingTimeEstimator", "CSVLogger", "JSONLLogger", "WandbLogger", "DDPStrategy",
           "DeepSpeedStrategy", "FSDP2Strategy", "SingleDeviceStrategy", "Strategy", "Trainer"]
