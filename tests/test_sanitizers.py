"""Host-code sanitizer run: the regex compiler and the threaded batch packer under
ASan+UBSan and TSan (tools/sanitize_host.sh, tools/native/selftest.cpp). CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
@pytest.mark.timeout(900)
def test_host_sanitizers_clean():
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize_host.sh"), "1500"], capture_output=True,
                       text=True, cwd=ROOT, timeout=850)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("OK (0 failures)") == 2
