"""Documentation hygiene: every `profiles/...` file that the docs, sources and
tools cite is a tracked file (tools/check_citations.py)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("git") is None or not os.path.isdir(os.path.join(ROOT, ".git")),
                    reason="needs the git checkout")
def test_profile_citations_resolve():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_citations.py")], cwd=ROOT,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
