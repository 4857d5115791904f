"""Training: CLI config, trainer engine, LR schedulers, metrics."""
from .config import ScaleTorchArguments, parse_args
from .lr_scheduler import available_schedulers, create_lr_scheduler, register_scheduler

__all__ = ["ScaleTorchArguments", "parse_args", "available_schedulers", "create_lr_scheduler",
           "register_scheduler"]
