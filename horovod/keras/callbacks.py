"""``horovod.keras.callbacks`` → :mod:`mivod.keras.callbacks`."""
from mivod.keras.callbacks import (BroadcastGlobalVariablesCallback,  # noqa: F401
                                   LearningRateScheduleCallback, LearningRateWarmupCallback,
                                   MetricAverageCallback)
