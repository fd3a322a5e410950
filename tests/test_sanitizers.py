"""Host runtime under sanitizers: the native self-test
(csrc/tests/host_selftest.cc -- LZ4, CRB, parsers, splits, the threaded
ordered reader, the workload pool under concurrent workers, the TCP van)
runs plain, under AddressSanitizer and under ThreadSanitizer, and must
report nothing. Host code only: GPU sanitizers are not used."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_selftest_plain():
    exe = os.path.join(ROOT, "bin", "native", "host_selftest")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "host_selftest: ok" in r.stdout, r.stderr[-3000:]


@pytest.mark.parametrize("kind", ["address", "thread", "undefined"])
def test_host_selftest_sanitized(kind, tmp_path):
    b = subprocess.run([sys.executable, os.path.join(ROOT, "build_native.py"), "--sanitize", kind],
                       capture_output=True, text=True, timeout=900)
    assert b.returncode == 0, b.stderr[-3000:]
    exe = b.stdout.strip().splitlines()[-1]
    env = dict(os.environ, TMPDIR=str(tmp_path),
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr
    assert "ERROR: AddressSanitizer" not in r.stderr
    assert "runtime error" not in r.stderr
    assert "host_selftest: ok" in r.stdout
