"""Step watchdog: turn a silent hang into a diagnosable, restartable failure.

The reference relies on the 180 s process-group timeout and ``--max-restarts=0``
(SURVEY.md §5.3).  A hung collective on RCCL may never return to Python, so
an in-loop check cannot see it.  ``StepWatchdog`` runs a daemon thread; the
training loop calls ``kick(step)`` once per step.  If no kick arrives within
``timeout_s`` the watchdog dumps every thread's Python stack (faulthandler)
plus the last step number, then calls ``on_timeout`` -- by default
``os._exit(EXIT_CODE)`` so ``torchrun --max-restarts N`` restarts the job and
``--auto_resume`` continues from the newest checkpoint.
"""
from __future__ import annotations

import faulthandler
import logging
import os
import sys
import threading
import time

logger = logging.getLogger(__name__)

EXIT_CODE = 75  # EX_TEMPFAIL: "try again"


def _default_on_timeout(info: str) -> None:
    sys.stderr.write(f"[watchdog] {info}; exiting with {EXIT_CODE} for a supervised restart\n")
    sys.stderr.flush()
    os._exit(EXIT_CODE)


class StepWatchdog:
    def __init__(self, timeout_s: float, on_timeout=None, poll_s: float | None = None):
        self.timeout_s = float(timeout_s)
        self.on_timeout = on_timeout or _default_on_timeout
        self.poll_s = poll_s if poll_s is not None else max(0.05, min(10.0, self.timeout_s / 10))
        self._last = time.monotonic()
        self._step = -1
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self.fired = False

    def start(self) -> "StepWatchdog":
        self._last = time.monotonic()
        self._thread = threading.Thread(target=self._run, name="st-watchdog", daemon=True)
        self._thread.start()
        return self

    def kick(self, step: int | None = None) -> None:
        self._last = time.monotonic()
        if step is not None:
            self._step = step

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            idle = time.monotonic() - self._last
            if idle > self.timeout_s and not self.fired:
                self.fired = True
                info = (f"no training progress for {idle:.1f}s (limit {self.timeout_s:.0f}s) after step "
                        f"{self._step}")
                logger.error(info)
                try:
                    faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                except Exception:  # pragma: no cover - stderr closed
                    pass
                self.on_timeout(info)
