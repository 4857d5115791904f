"""Utilities: device/FLOPS registry, MFU, checkpoints, logging, monitoring."""
