"""Optimizers: fused LAMB / LARC-SGD on flat buffers, LR schedules, PerformanceEMA, CollaborativeOptimizer."""
from .collaborative import CollaborationState, CollaborativeOptimizer, TrainingState
from .lamb import (FusedLamb, FusedLarcSGD, LambdaScheduler, LinearWarmupCosineAnnealingLR,
                   get_linear_schedule_with_warmup)
from .performance_ema import PerformanceEMA

__all__ = ["CollaborationState", "CollaborativeOptimizer", "TrainingState", "FusedLamb", "FusedLarcSGD",
           "LambdaScheduler", "LinearWarmupCosineAnnealingLR", "get_linear_schedule_with_warmup", "PerformanceEMA"]
