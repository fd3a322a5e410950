#!/usr/bin/env python3
"""End-to-end throughput from FILES through the whole PS stack -- the path a
user of the reference's Criteo tutorial runs (doc/tutorial/criteo_kaggle.rst:
`dmlc_local.py -n W -s S bin/linear.dmlc ...`, published 1.85 M examples/s):
tracker -> scheduler (workload pool over virtual file parts) -> worker
(parallel text parser -> minibatches -> H2D -> localize -> pull -> loss ->
push -> FTRL) -> progress table.

The Criteo-format text (label, 13 integer, 26 categorical fields) is
synthesised with fixed-width fields by vectorised numpy (no dataset is
reachable here), optionally converted to CRB with bin/convert.dmlc, and
trained for one data pass. Throughput = examples / wall time of the job's
training pass, read from the scheduler's progress table.

    python benchmarks/bench_e2e.py [--rows 2000000] [--files 4] [--model linear|difacto]
                                   [--format criteo|crb] [-n 1]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HEX = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)
DIG = np.frombuffer(b"0123456789", dtype=np.uint8)


def criteo_text(nrows, seed):
    """nrows lines of fixed-width Criteo TSV: 1-char label, 13 4-digit ints,
    26 8-hex categoricals (power-law values so ids repeat like real data)."""
    rng = np.random.default_rng(seed)
    width = 1 + 13 * 5 + 26 * 9 + 1
    buf = np.empty((nrows, width), dtype=np.uint8)
    lab = (rng.random(nrows) < 0.25).astype(np.uint8)
    buf[:, 0] = DIG[lab]
    col = 1
    for _ in range(13):
        v = np.minimum((rng.pareto(1.2, nrows) * 3).astype(np.int64), 9999)
        buf[:, col] = 9  # tab
        for d in range(4):
            buf[:, col + 4 - d] = DIG[(v // 10 ** d) % 10]
        col += 5
    for f in range(26):
        card = int(10 ** rng.uniform(1, 6.5))
        v = (np.minimum(rng.pareto(1.1, nrows) * 2, card - 1).astype(np.int64) * 2654435761
             + f * 97) & 0xFFFFFFFF
        buf[:, col] = 9
        for d in range(8):
            buf[:, col + 8 - d] = HEX[(v >> (4 * d)) & 15]
        col += 9
    buf[:, col] = 10  # newline
    return buf.tobytes()


def _run_job(cmd, work, vper):
    """One run of the job; the training pass(es) run from the first
    "Training: iter = 0" line to the "Validating" / "Hit max" line that
    follows the last pass, and their examples are the last progress-table
    row of each pass (the table restarts every pass)."""
    t1 = time.time()
    proc = subprocess.Popen(cmd, cwd=work, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                            text=True, bufsize=1)
    lines, stamps = [], []
    for line in proc.stdout:
        lines.append(line)
        stamps.append(time.time())
    err = proc.stderr.read()
    rc = proc.wait()
    wall = time.time() - t1
    out = "".join(lines)
    if rc != 0:
        sys.stderr.write(out[-3000:] + err[-3000:])
        raise SystemExit(rc)
    is_row = [bool(re.match(r"^\s*[\d.]+\s+[\d.e+]+\s+[\d.e+]+", l)) for l in lines]
    # each pass: from its "Training: iter = k" line to the next stage line
    # ("Validating" -- printed after every pass, with or without val_data --
    # or "Hit max"); the examples are its table's last row
    sec, ttl, vttl, v_start, v_end = 0.0, 0.0, 0.0, None, None
    last_row, phase, p_start = None, None, None
    for i, l in enumerate(lines):
        stage = l.startswith(("Training: iter", "Validating", "Hit max"))
        if stage:
            if phase == "train":
                sec += stamps[i] - p_start
                ttl += last_row or 0.0
            elif phase == "val":
                vttl += last_row or 0.0
                if vper:
                    v_end = stamps[i]
            last_row = None
            phase = None
        if l.startswith("Training: iter"):
            phase, p_start = "train", stamps[i]
        elif l.startswith("Validating"):
            phase = "val"
            if v_start is None:
                v_start = stamps[i]
        elif is_row[i] and phase is not None:
            last_row = float(l.split()[1])
    print(out[-1500:], file=sys.stderr)
    for l in err.splitlines():  # the workers' per-pass stage summaries
        if "minibatches" in l or "[ingest]" in l:
            print(l, file=sys.stderr)
    return {"value": ttl / sec if sec > 0 else None, "examples": ttl, "train_sec": sec,
            "job_wall_sec": wall,
            "val_examples_per_s": (vttl / (v_end - v_start)) if (vper and v_start and v_end)
            else None, "val_examples": vttl if vper else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--files", type=int, default=4)
    ap.add_argument("--model", default="linear", choices=["linear", "difacto"])
    ap.add_argument("--format", default="criteo", choices=["criteo", "crb"])
    ap.add_argument("-n", type=int, default=1, help="workers (one GPU each)")
    ap.add_argument("--minibatch", type=int, default=100000)
    ap.add_argument("--val-rows", type=int, default=0,
                    help="also write this many validation rows (val_data) and time the "
                         "validation pass (the reference log's 0.93 M ex/s)")
    ap.add_argument("--rand-shuffle", type=int, default=10,
                    help="shuffle buffer in minibatches (the reference default is 10)")
    ap.add_argument("--passes", type=int, default=1,
                    help="data passes (max_data_pass): a timed region of several seconds "
                         "over files that fit the box")
    ap.add_argument("--repeat", type=int, default=1,
                    help="run the job this many times over the same files and report the "
                         "median and the spread")
    ap.add_argument("--dir", default=None)
    ap.add_argument("--reuse", action="store_true",
                    help="keep the data files already in --dir (A/B runs over the same files)")
    args = ap.parse_args()
    if args.passes > 1 and args.val_rows:
        raise SystemExit("--passes > 1 with --val-rows is not supported (validation per pass)")
    work = args.dir or tempfile.mkdtemp(prefix="wh_e2e_")
    os.makedirs(work, exist_ok=True)
    t0 = time.time()
    per = args.rows // args.files
    for i in range(args.files):
        p = os.path.join(work, "train-part_%d.txt" % i)
        if args.reuse and os.path.exists(p[:-4] + (".crb" if args.format == "crb" else ".txt")):
            continue
        with open(p, "wb") as f:
            f.write(criteo_text(per, 100 + i))
        if args.format == "crb":
            subprocess.run([os.path.join(ROOT, "bin", "convert.dmlc"),
                            "-data_in", p, "-data_out", p[:-4] + ".crb", "-format_in", "criteo",
                            "-format_out", "crb"], check=True)
            os.remove(p)
    vper = args.val_rows // args.files if args.val_rows else 0
    for i in range(args.files if vper else 0):
        if args.reuse and os.path.exists(os.path.join(work, "val-part_%d.txt" % i)):
            continue
        with open(os.path.join(work, "val-part_%d.txt" % i), "wb") as f:
            f.write(criteo_text(vper, 900 + i))
    gen_s = time.time() - t0
    pattern = os.path.join(work, "train-part_.*\\.%s" % ("crb" if args.format == "crb" else "txt"))
    conf = os.path.join(work, "job.conf")
    with open(conf, "w") as f:
        f.write('train_data = "%s"\ndata_format = "%s"\nminibatch = %d\nmax_data_pass = %d\n'
                "print_sec = 1\nrand_shuffle = %d\n" % (pattern, args.format, args.minibatch,
                                                   args.passes, args.rand_shuffle))
        if vper:
            f.write('val_data = "%s"\n' % os.path.join(work, "val-part_.*\\.txt"))
        if args.model == "linear":
            f.write("lambda_l1 = 4\nlr_eta = 0.1\n")
        else:
            f.write("lr_eta = 0.01\nembedding {\n  dim = 64\n  threshold = 100\n"
                    "  lambda_l2 = 1\n  lr_eta = 0.01\n}\n")
    binp = os.path.join(ROOT, "bin", "%s.dmlc" % args.model)
    cmd = [sys.executable, os.path.join(ROOT, "tracker", "dmlc_local.py"), "-n", str(args.n),
           "-s", str(args.n), binp, conf]
    runs = [_run_job(cmd, work, vper) for _ in range(max(1, args.repeat))]
    vals = sorted(r["value"] for r in runs if r["value"])
    med = vals[len(vals) // 2] if vals else None
    r = runs[-1]
    print(json.dumps({
        "metric": "end-to-end examples/sec from %s files, %s.dmlc, %d worker(s)" % (
            args.format, args.model, args.n),
        "value": med, "unit": "examples/s",
        "runs": [round(x["value"] / 1e6, 2) if x["value"] else None for x in runs],
        "runs_unit": "M examples/s", "spread_min": vals[0] if vals else None,
        "spread_max": vals[-1] if vals else None,
        "examples": r["examples"], "train_sec": r["train_sec"], "job_wall_sec": r["job_wall_sec"],
        "datagen_sec": gen_s, "passes": args.passes,
        "reference_linear_published": 1.85e6,
        "val_examples_per_s": r["val_examples_per_s"], "val_examples": r["val_examples"],
        "reference_linear_val_published": 0.93e6,
        "config": {"rows": args.rows, "files": args.files, "minibatch": args.minibatch,
                   "val_rows": args.val_rows,
                   "rand_shuffle": args.rand_shuffle,
                   "device_parse": os.environ.get("WH_DEVICE_PARSE", "1") != "0"},
    }))


if __name__ == "__main__":
    main()
