"""Static check: no undefined global names anywhere in the package (GPU-only code paths are not executed by the
CPU suite, so a deleted module-level name would otherwise only surface on the GPU box)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_undefined_names():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "lint_names.py"),
                        os.path.join(ROOT, "deeplearning4j_amd"), os.path.join(ROOT, "tools")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
