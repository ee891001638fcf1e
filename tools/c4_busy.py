"""C4's shape alone (bench.c4_rate: s-seg 640 f32, one frame per step, three in flight) for a kernel trace, and
the GPU-busy fraction of a trace: is the shape bound by the GPU or by the host issuing it?
  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c4 -o c4 -- python tools/c4_busy.py run
  python tools/c4_busy.py busy gpurun_out/c4/c4_kernel_trace.csv"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def busy(path):
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(path))))
    rows = rows[len(rows) // 2:]  # the second half: steady state of the timed steps
    t0, t1 = rows[0][0], max(e for _, e in rows)
    covered, cs, ce = 0, None, None
    for s, e in rows:
        if cs is None or s > ce:
            if cs is not None:
                covered += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    covered += ce - cs
    ksum = sum(e - s for s, e in rows)
    print(json.dumps({"window_us": round((t1 - t0) / 1e3, 1), "busy_frac": round(covered / (t1 - t0), 3),
                      "kernel_sum_over_window": round(ksum / (t1 - t0), 3), "kernels": len(rows)}))


def run():
    import torch
    import bench
    sys.argv = ["bench.py", "--steps", "20"]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    print(json.dumps(bench.c4_rate(args, dev, 0, 1, False)))


if __name__ == "__main__":
    busy(sys.argv[2]) if sys.argv[1] == "busy" else run()
