"""The RCCL communicator's watchdog/abort race: a failed
communicator must never be aborted (ncclCommAbort frees it) while a host call
on another thread still holds the handle.  The handle-retirement state machine
of csrc/comm/communicator.h lives in the HIP-free header csrc/comm/retirable.h;
this builds a threaded C++ driver against it with g++ and runs it on the CPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_retire_waits_for_inflight_calls(tmp_path):
    exe = tmp_path / "retirable_test"
    src = os.path.join(ROOT, "tests", "unit", "native", "retirable_test.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-pthread", "-fsanitize=thread", "-I", os.path.join(ROOT, "csrc"),
                    src, "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "retirable: ok" in out.stdout
