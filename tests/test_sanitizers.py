"""The threaded / bigint host modules run clean under ASan+UBSan and (loader) TSan
(tools/sanitize_host.py).  Needs g++ with the sanitizer runtimes and the
image's libpng / GMP / libhdf5."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(shutil.which("g++") is None or not os.path.exists("/opt/conda/include/gmp.h"),
                                reason="no host toolchain / libraries for the sanitizer builds")


@pytest.mark.timeout(900)
@pytest.mark.parametrize("kind", ["address", "thread"])
def test_host_modules_clean_under_sanitizer(kind):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sanitize_host.py"), kind], cwd=ROOT,
                       capture_output=True, text=True, timeout=850)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert "instrumented:" in r.stdout and " passed" in r.stdout
