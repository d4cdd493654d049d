"""engine._capturing: around every hipGraph capture the communicator's
watchdog stops polling and the cyclic GC is off (either could issue a HIP call
mid-capture and invalidate it); both come back afterwards, also on error."""
import gc
import os
import shutil
import subprocess

import pytest

from torch_distlearn_amd.engine import _capturing

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_native_pause_waits_for_a_running_poll(tmp_path):
    """The native half of the guard: the communicator's
    set_paused(True) returns only once no watchdog poll is running -- a poll
    already past its pause check, and the part of a poll run without the lock,
    finish first -- and no poll starts until resumed (csrc/comm/pause_gate.h,
    the handshake RcclCommunicator uses; C++ driver under ThreadSanitizer)."""
    exe = tmp_path / "pause_gate_test"
    src = os.path.join(ROOT, "tests", "unit", "native", "pause_gate_test.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-pthread", "-fsanitize=thread", "-I", os.path.join(ROOT, "csrc"),
                    src, "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "pause_gate: ok" in out.stdout
