"""Run the linear demo (learn/linear/guide/demo.conf) under several step /
ingest modes and print the validation lines (GPU debugging aid)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CODE = ("import sys; sys.path.insert(0, %r)\n"
        "from wormhole_amd.apps.ps_app import main\n"
        "main(%r, [%r, 'rand_shuffle=0'] + sys.argv[1:])\n")
app = sys.argv[1] if len(sys.argv) > 1 else "linear"
conf = "learn/%s/guide/demo.conf" % app
modes = [("cpu", {"WH_DEVICE": "cpu"}), ("gpu", {"WH_DEVICE": "auto"}),
         ("gpu-hostparse", {"WH_DEVICE": "auto", "WH_DEVICE_PARSE": "0"}),
         ("gpu-deterministic", {"WH_DEVICE": "auto", "WH_DETERMINISTIC": "1"})]
work = "/tmp/demo_modes"
os.makedirs(work, exist_ok=True)
if not os.path.exists(os.path.join(work, "learn")):
    os.symlink(os.path.join(ROOT, "learn"), os.path.join(work, "learn"))
for name, env in modes:
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", CODE % (ROOT, app, conf)] + sys.argv[2:], cwd=work,
                       env=e, capture_output=True, text=True, timeout=240)
    lines = [l for l in r.stdout.splitlines() if l.strip()[:1].isdigit()]
    print("==", name, "rc", r.returncode)
    for l in lines:
        print("  ", l)
    if r.returncode:
        print(r.stderr[-2000:])
