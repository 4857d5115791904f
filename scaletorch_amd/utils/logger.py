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


class _DeviceTelemetry:
    """Temperature / power / utilisation of this rank's GPU through ``amdsmi`` (ROCm's
    SMI library) when it is importable; every read is best-effort (a missing metric
    is simply absent).  Reference: the optional NVML block of
    scaletorch/utils/monitor.py:34-292."""

    def __init__(self, device_index: int = 0):
        self.handle = None
        self.amdsmi = None
        try:
            import amdsmi

            amdsmi.amdsmi_init()
            handles = amdsmi.amdsmi_get_processor_handles()
            if handles:
                self.amdsmi = amdsmi
                self.handle = handles[min(device_index, len(handles) - 1)]
        except Exception:  # no SMI, no permission, no GPU: telemetry off
            self.handle = None

    def read(self) -> dict:
        if self.handle is None:
            return {}
        a, h, out = self.amdsmi, self.handle, {}
        for key, fn in (("gpu_temp_c", lambda: a.amdsmi_get_temp_metric(h, a.AmdSmiTemperatureType.HOTSPOT,
                                                                          a.AmdSmiTemperatureMetric.CURRENT)),
                        ("gpu_power_w", lambda: a.amdsmi_get_power_info(h).get("current_socket_power")),
                        ("gpu_busy_pct", lambda: a.amdsmi_get_gpu_activity(h).get("gfx_activity"))):
            try:
                v = fn()
                if isinstance(v, (int, float)):
                    out[key] = float(v)
            except Exception:
                pass
        return out


class PerformanceMonitor:
    """Per-iteration throughput, memory and device telemetry WITHOUT forcing device
    synchronisation.

    Iterations are bracketed by events recorded on the current (compute) stream;
    a step's time is the distance between consecutive end events, i.e. the steady
    step period on the device timeline, so work a side stream overlaps into the
    next step (optimizer update, ZeRO-1 gathers) is NOT forced to finish first --
    ``torch.cuda.synchronize()`` per step (which waits for every stream) would
    remove exactly that overlap.  Records are resolved lazily: when their end event
    has completed, or when the caller asks (``sync=True``, at logging steps, where
    the loss read synchronises anyway).  Averages use ring buffers of ``window``
    steps and exclude warm-up; telemetry (allocator fragmentation, GPU temperature
    / power / activity via amdsmi, host CPU / RSS via psutil) is sampled every
    ``telemetry_interval`` steps.  Reference: scaletorch/utils/monitor.py:34-292.
    """

    def __init__(self, warmup_steps: int = 2, window: int = 1000, rank: int = 0, telemetry_interval: int = 10,
                 device_index: int | None = None):
        self.warmup, self.rank = warmup_steps, rank
        self.extra: dict = {}  # static / run-level entries merged into summary() (comm volume, PP bubble)
        self.times = deque(maxlen=window)
        self.tokens = deque(maxlen=window)
        self.telemetry = {}
        self.records = []
        self.step = 0
        self.telemetry_interval = max(1, telemetry_interval)
        self._cuda = torch.cuda.is_available()
        self._pending = []  # (record, start_event, end_event)
        self._last_end = None
        self._t0 = None
        self._last_wall = None
        self._smi = None
        if self._cuda:
            self._smi = _DeviceTelemetry(torch.cuda.current_device() if device_index is None else device_index)

    def start_iteration(self) -> None:
        if self._cuda:
            self._start_ev = torch.cuda.Event(enable_timing=True)
            self._start_ev.record()
        else:
            self._t0 = time.perf_counter()

    def end_iteration(self, tokens: int, extra: dict | None = None, sync: bool = False) -> dict:
        self.step += 1
        rec = {"step": self.step, "tokens": tokens}
        if extra:
            rec.update(extra)
        if self._cuda:
            end = torch.cuda.Event(enable_timing=True)
            end.record()
            # period from the previous step's end (steady state) or from this step's start
            begin = self._last_end if self._last_end is not None else self._start_ev
            self._pending.append((rec, begin, end))
            self._last_end = end
        else:
            now = time.perf_counter()
            begin = self._last_wall if self._last_wall is not None else self._t0
            self._last_wall = now
            self._finish(rec, now - begin)
        if self.step % self.telemetry_interval == 0 or self.step == 1:
            rec.update(self._sample_telemetry())
        self.resolve(block=sync)
        self.records.append(rec)
        return rec

    def _finish(self, rec: dict, dt: float) -> None:
        rec["step_time_s"] = dt
        rec["tokens_per_s"] = rec["tokens"] / dt if dt > 0 else 0.0
        if rec["step"] > self.warmup:
            self.times.append(dt)
            self.tokens.append(rec["tokens"])

    def resolve(self, block: bool = False) -> None:
        """Fill in the step times whose end event completed (all of them if ``block``)."""
        while self._pending:
            rec, begin, end = self._pending[0]
            if not block and not end.query():
                break
            end.synchronize()
            self._finish(rec, begin.elapsed_time(end) / 1e3)
            self._pending.pop(0)

    def _sample_telemetry(self) -> dict:
        t = {}
        if self._cuda:
            alloc, reserved = torch.cuda.memory_allocated(), torch.cuda.memory_reserved()
            t.update(mem_allocated_gb=alloc / 1e9, mem_reserved_gb=reserved / 1e9,
                     mem_peak_gb=torch.cuda.max_memory_allocated() / 1e9,
                     mem_fragmentation=(1.0 - alloc / reserved) if reserved else 0.0)
            if self._smi is not None:
                t.update(self._smi.read())
        try:
            import psutil

            p = psutil.Process()
            t.update(cpu_percent=psutil.cpu_percent(interval=None), host_rss_gb=p.memory_info().rss / 1e9)
        except Exception:
            pass
        for k, v in t.items():
            self.telemetry.setdefault(k, deque(maxlen=self.times.maxlen)).append(v)
        return t

    def summary(self) -> dict:
        self.resolve(block=True)
        if not self.times:
            return {}
        ts = sorted(self.times)
        total_t = sum(self.times)
        out = {"steps_measured": len(ts), "mean_step_s": total_t / len(ts), "median_step_s": ts[len(ts) // 2],
               "tokens_per_s": sum(self.tokens) / total_t}
        out.update(self.extra)
        for k, v in self.telemetry.items():
            if v:
                out[f"avg_{k}"] = sum(v) / len(v)
                out[f"max_{k}"] = max(v)
        return out

    def dump(self, out_dir: str = ".") -> str:
        self.resolve(block=True)
        os.makedirs(out_dir, exist_ok=True)
        path = os.path.join(out_dir, f"performance_logs_{self.rank}_{int(time.time())}.json")
        with open(path, "w") as f:
            json.dump({"summary": self.summary(), "records": self.records}, f, indent=1)
        return path
