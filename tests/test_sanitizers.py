"""Host-code memory safety: the native runtime's parsers run under ASan + UBSan on
valid, truncated and bit-flipped inputs (tools/sanitize_rt.sh)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(300)
@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_under_asan_ubsan(tmp_path):
    r = subprocess.run([os.path.join(REPO, "tools", "sanitize_rt.sh"), str(tmp_path)], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=280)
    assert r.returncode == 0, r.stdout
    assert "rt_selftest: ok" in r.stdout
