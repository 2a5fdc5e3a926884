"""Training driver (reference: training/)."""
from .training import AdamOptimizer, Training

__all__ = ["AdamOptimizer", "Training"]
