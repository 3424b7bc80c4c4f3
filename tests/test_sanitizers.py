"""Host-code sanitizers (SURVEY.md §5 "Race detection / sanitizers"): the transport, ring and API
C++ built with ThreadSanitizer / AddressSanitizer / UBSan (-Xarch_host only) and driven through
dccl_cli on host buffers with 1-8 thread-ranks.  Any report fails the run (halt_on_error)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("kind", ["thread", "address", "undefined"])
def test_host_sanitizer(kind):
    if not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("make") is None:
        pytest.skip("no hipcc")
    p = subprocess.run([os.path.join(ROOT, "tools", "sanitize_host.sh"), kind], capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert f"sanitize_host({kind}): clean" in p.stdout
