"""bin/_launch.py run(): the app launchers' exit path (flush, then os._exit
with main's code) keeps the codes and messages a plain sys.exit(main())
would give."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r"""
import sys
sys.path.insert(0, {bin!r})
import _launch
kind = sys.argv[1]
def main(x):
    print("out " + x)
    sys.stderr.write("err " + x + "\n")
    if kind == "int":
        return 3
    if kind == "none":
        return None
    if kind == "str":
        raise SystemExit("stopped: " + x)
    if kind == "raise":
        raise ValueError("boom " + x)
    if kind == "exit0":
        raise SystemExit(0)
_launch.run(main, "a")
print("not reached")
"""


@pytest.mark.parametrize("kind,code,err", [("int", 3, None), ("none", 0, None),
                                           ("str", 1, "stopped: a"), ("raise", 1, "ValueError: boom a"),
                                           ("exit0", 0, None)])
def test_launch_run_exit_codes(tmp_path, kind, code, err):
    script = tmp_path / "app.py"
    script.write_text(_SCRIPT.format(bin=os.path.join(ROOT, "bin")))
    r = subprocess.run([sys.executable, str(script), kind], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == code, (r.stdout, r.stderr)
    # buffered stdout is flushed before the process leaves; nothing after run()
    assert r.stdout.splitlines() == ["out a"]
    assert "err a" in r.stderr
    if err:
        assert err in r.stderr
