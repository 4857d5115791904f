"""Rank-aware logging + per-iteration performance monitor.

Reference: scaletorch/utils/logger_utils.py:18-149 (colored, rank-0 stream handler)
and PerformanceMonitor (scaletorch/utils/monitor.py:34-292: per-iteration wall
time, tokens/s, memory, JSON dump).  The monitor here times the FULL step
(the trainer calls it around fwd+bwd+comm+clip+optimizer) and excludes warm-up
steps from its averages.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time
from collections import deque

import torch

_COLORS = {"DEBUG": "\033[36m", "INFO": "\033[32m", "WARNING": "\033[33m", "ERROR": "\033[31m",
           "CRITICAL": "\033[35m"}


class _Fmt(logging.Formatter):
    def __init__(self, color: bool):
        super().__init__("[%(asctime)s] [%(levelname)s] [rank %(rank)s] %(name)s: %(message)s", "%H:%M:%S")
        self.color = color

    def format(self, record):
        record.rank = os.environ.get("RANK", "0")
        s = super().format(record)
        if self.color and record.levelname in _COLORS:
            s = _COLORS[record.levelname] + s + "\033[0m"
        return s


def get_logger(name: str = "scaletorch_amd", level: int = logging.INFO, all_ranks: bool = False) -> logging.Logger:
    log = logging.getLogger(name)
    if getattr(log, "_st_configured", False):
        return log
    rank = int(os.environ.get("RANK", "0"))
    h = logging.StreamHandler(sys.stdout)
    h.setFormatter(_Fmt(color=sys.stdout.isatty()))
    log.addHandler(h)
    log.setLevel(level if (rank == 0 or all_ranks) else logging.ERROR)
    log.propagate = False
    log._st_configured = True
    return log


class PerformanceMonitor:
    def __init__(self, warmup_steps: int = 2, window: int = 1000, rank: int = 0):
        self.warmup, self.rank = warmup_steps, rank
        self.times = deque(maxlen=window)
        self.tokens = deque(maxlen=window)
        self.records = []
        self._t0 = None
        self.step = 0

    def start_iteration(self) -> None:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self._t0 = time.perf_counter()

    def end_iteration(self, tokens: int, extra: dict | None = None) -> dict:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dt = time.perf_counter() - self._t0
        self.step += 1
        rec = {"step": self.step, "step_time_s": dt, "tokens_per_s": tokens / dt if dt > 0 else 0.0}
        if torch.cuda.is_available():
            rec.update(mem_allocated_gb=torch.cuda.memory_allocated() / 1e9,
                       mem_reserved_gb=torch.cuda.memory_reserved() / 1e9,
                       mem_peak_gb=torch.cuda.max_memory_allocated() / 1e9)
        if extra:
            rec.update(extra)
        self.records.append(rec)
        if self.step > self.warmup:
            self.times.append(dt)
            self.tokens.append(tokens)
        return rec

    def summary(self) -> dict:
        if not self.times:
            return {}
        ts = sorted(self.times)
        total_t = sum(self.times)
        return {"steps_measured": len(ts), "mean_step_s": total_t / len(ts), "median_step_s": ts[len(ts) // 2],
                "tokens_per_s": sum(self.tokens) / total_t}

    def dump(self, out_dir: str = ".") -> str:
        os.makedirs(out_dir, exist_ok=True)
        path = os.path.join(out_dir, f"performance_logs_{self.rank}_{int(time.time())}.json")
        with open(path, "w") as f:
            json.dump({"summary": self.summary(), "records": self.records}, f, indent=1)
        return path
