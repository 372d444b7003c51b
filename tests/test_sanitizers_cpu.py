"""Host sanitizers over the native runtime: the C++ runtime
(TF bundle, TFRecord/tfevents, TCP store, blocking queue, libsvm parser) is
rebuilt with ASan+UBSan and with TSan and driven through concurrent and
edge-case paths (scripts/asan_runtime.py).  Building two sanitizer modules
takes a few minutes, so this runs when DTF_SANITIZERS=1."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(os.environ.get("DTF_SANITIZERS") != "1", reason="set DTF_SANITIZERS=1")


@pytest.mark.parametrize("mode", ["asan", "tsan"])
def test_runtime_under_sanitizer(mode):
    args = [sys.executable, os.path.join(REPO, "scripts", "asan_runtime.py")] + (["--tsan"] if mode == "tsan" else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=1500)
    assert r.returncode == 0 and "exercise: clean" in r.stdout, (r.stdout + r.stderr)[-4000:]
