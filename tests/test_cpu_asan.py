"""SURVEY.md §5 sanitizers, host side: the C ABI built with the host code under AddressSanitizer
(tools/asan_abi.py) and driven through every entry point declared in include/ivit.h with argument
patterns that validation must reject or that must be no-ops (zero / negative sizes, NULL pointers),
the workspace queries at the product's shapes, and the kernel-timing bookkeeping with real host
buffers. Each call runs in its own forked child, so a failure names every offending entry point.
CPU only: no kernel runs (a first build compiles csrc/ once more, ~2.5 min; later runs are
incremental)."""
import os
import shutil
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
TOOL = os.path.join(HERE, "..", "tools", "asan_abi.py")

pytestmark = pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not available")


@pytest.mark.timeout(900)
def test_abi_validation_clean_under_asan():
    r = subprocess.run([sys.executable, TOOL], capture_output=True, text=True, timeout=880)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out
    assert "0 failed" in out and "no AddressSanitizer report" in out
