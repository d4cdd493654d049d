"""engine._capturing: around every hipGraph capture the communicator's
watchdog stops polling and the cyclic GC is off (either could issue a HIP call
mid-capture and invalidate it); both come back afterwards, also on error."""
import gc

import pytest

from torch_distlearn_amd.engine import _capturing


class _Comm:
    def __init__(self):
        self.calls = []

    def pause_watch(self, paused):
        self.calls.append(paused)


def test_capturing_pauses_watchdog_and_gc():
    assert gc.isenabled()
    c = _Comm()
    with _capturing(c):
        assert not gc.isenabled() and c.calls == [True]
    assert gc.isenabled() and c.calls == [True, False]


def test_capturing_restores_on_error_and_without_watchdog():
    c = _Comm()
    with pytest.raises(RuntimeError):
        with _capturing(c):
            raise RuntimeError("capture failed")
    assert gc.isenabled() and c.calls == [True, False]
    with _capturing(object()):  # a communicator without a watchdog (gloo)
        assert not gc.isenabled()
    assert gc.isenabled()
    gc.disable()  # a caller that had the GC off keeps it off
    try:
        with _capturing(c):
            pass
        assert not gc.isenabled()
    finally:
        gc.enable()
