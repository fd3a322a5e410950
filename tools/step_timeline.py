#!/usr/bin/env python3
"""Print one training step's kernel timeline (start offset, gap before,
duration, queue) from a rocprofv3 kernel trace; steps are delimited by a
marker kernel (default: the synthetic-data generator). The summary line
gives the step span, the summed kernel time and the time NO kernel ran
(idle: the union of the kernel intervals subtracted from the span).

    python tools/step_timeline.py gpurun_out/TAG/prof [marker] [step_from_end]
"""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_synth_criteo"
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    path = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    i0, i1 = idx[-back], idx[-back + 1]
    t0 = int(rows[i0]["Start_Timestamp"])
    t1 = int(rows[i1]["Start_Timestamp"])
    prev = t0
    busy = 0.0
    covered, cur_s, cur_e = 0, None, None
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += (e - s) / 1e3
        q = r.get("Queue_Id", r.get("Stream_Id", "?"))
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        print("%8.1f gap %6.1f dur %6.1f q%-3s %s" % ((s - t0) / 1e3, (s - prev) / 1e3,
                                                     (e - s) / 1e3, q, name[:70]))
        prev = e
        e = min(e, t1)
        if cur_s is None or s > cur_e:
            if cur_s is not None:
                covered += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_s is not None:
        covered += cur_e - cur_s
    total = (t1 - t0) / 1e3
    print("step %.1f us, kernels %d, summed %.1f us, idle %.1f us" %
          (total, i1 - i0, busy, total - covered / 1e3))


if __name__ == "__main__":
    main()
