"""Fused flat-arena optimizers (hand-written gfx950 kernels on GPU)."""
from .fused import (Arena, FusedAdadelta, FusedAdam, FusedAdamW, FusedLARS, FusedOptimizer,
                    FusedSGD)

__all__ = ["Arena", "FusedOptimizer", "FusedSGD", "FusedAdam", "FusedAdamW", "FusedAdadelta",
           "FusedLARS"]
