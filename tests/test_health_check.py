"""Trainer.health_check reads the error word of every xGMI communicator the run uses:
the EP exchange's too (round 6: a timed-out EP exchange left its rows unwritten and
nothing polled it).  Fake communicators stand in for the IPC ones (CPU)."""
from __future__ import annotations

import types

import pytest


class _Comm:
    def __init__(self, bad: bool):
        self.bad = bad
        self.checked = 0

    def check(self):
        self.checked += 1
        if self.bad:
            raise RuntimeError("xgmi collective: a peer did not arrive")


def _trainer_stub():
    from scaletorch_amd.trainer.engine import Trainer

    t = Trainer.__new__(Trainer)
    t.args = types.SimpleNamespace(fused_lm_head=False)
    return t


def test_health_check_polls_ep_communicators(monkeypatch):
    from scaletorch_amd.models import moe

    good, bad = _Comm(False), _Comm(True)
    monkeypatch.setattr(moe, "_EP_XGMI", {1: good})
    _trainer_stub().health_check()
    assert good.checked == 1
    monkeypatch.setattr(moe, "_EP_XGMI", {1: good, 2: bad})
    with pytest.raises(RuntimeError, match="did not arrive"):
        _trainer_stub().health_check()


def test_check_xgmi_polls_the_pair_path(monkeypatch):
    from scaletorch_amd.parallel import tensor_parallel as tp

    bad = _Comm(True)
    monkeypatch.setattr(tp, "_XGMI", {})
    monkeypatch.setattr(tp, "_PAIR", [types.SimpleNamespace(comm=bad)])
    with pytest.raises(RuntimeError, match="did not arrive"):
        tp.check_xgmi()
