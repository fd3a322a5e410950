"""WH_DETERMINISTIC=1: two fresh processes training the same
DiFacto minibatches produce bitwise-identical progress sums and models (the
hash + stable-sort localize, and hot keys' gradient chunks summed in
occurrence order instead of float atomics). The default (fast) mode agrees
with it to float tolerance."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _run(env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(HERE, "_det_run.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("DIGEST")][-1].split()
    return line[1], float(line[3])


def test_deterministic_bitwise_repeat():
    a, la = _run({"WH_DETERMINISTIC": "1"})
    b, lb = _run({"WH_DETERMINISTIC": "1"})
    assert a == b, (la, lb)
    _, lf = _run({"WH_DETERMINISTIC": "0"})
    assert abs(lf - la) < 1e-4 * abs(la)
