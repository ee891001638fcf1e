#!/usr/bin/env python
"""Summarise rocprofv3 output of a bench.py run for profiles/.

  stats  <kernel_stats.csv> <out.json>
      per-family sums of the --kernel-trace --stats summary; the conv family (conv0/0_f32/0_f32m/2/3/3t/3u-3x/4/_dn/_patch/_wp, c2f, stem, pw
      kernels: every launch of the YOLOv8-seg forward's GEMMs) gives the average launch duration that
      bench.py's roofline.avg_launch_us must agree with.
  agree  <kernel_trace.csv> <bench_under_rocprof.json> <out.json> [launches_per_forward]
      the conv-family launches of the trace in dispatch order, cut into forwards, averaged per forward;
      the forwards after the warm-up and before the isolated tail are the timed region whose average must
      agree with the bench line's roofline.avg_launch_us (and the last three with isolated_avg_launch_us).
  traffic <fetch_counter_collection.csv> <write_counter_collection.csv> <key> <out.json>
      HBM bytes per conv launch from two separate --pmc passes (FETCH_SIZE, WRITE_SIZE), corrected as
      MI355X_MICROARCH.md §HBM prescribes for gfx950: both counters are in KiB; FETCH_SIZE reports half
      the bytes of a wide (16 B/lane) coalesced read, so it is doubled; WRITE_SIZE is exact for 16-byte
      stores.  Merged into <out.json> under <key> (bench.py reads profiles/conv_traffic.json).
"""
from __future__ import annotations

import csv
import json
import os
import re
import sys

CONV_RE = re.compile(r"(conv(0|2|3|4|8|3h|3t|3q|_dn|_patch|0_f32|0_f32m)?|c2f|stem|stem32|pw)_kernel")


def family(name: str) -> str:
    m = re.search(r"(\w+_kernel)", name)
    return m.group(1) if m else name[:60]


def stats(path: str, out: str) -> dict:
    fam = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            k = family(row["Name"])
            d = fam.setdefault(k, {"calls": 0, "total_ns": 0.0})
            d["calls"] += int(row["Calls"])
            d["total_ns"] += float(row["TotalDurationNs"])
    for d in fam.values():
        d["avg_us"] = round(d["total_ns"] / d["calls"] / 1e3, 3)
    conv = {"calls": 0, "total_ns": 0.0}
    for k, d in fam.items():
        if CONV_RE.search(k):
            conv["calls"] += d["calls"]
            conv["total_ns"] += d["total_ns"]
    conv["avg_us"] = round(conv["total_ns"] / max(conv["calls"], 1) / 1e3, 3)
    res = {"source": os.path.basename(path), "conv_family": conv,
           "families": dict(sorted(fam.items(), key=lambda kv: -kv[1]["total_ns"]))}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    return res


def agree(trace: str, bench_json: str, out: str, per_fwd: int = 58) -> dict:
    rows = []
    with open(trace) as f:
        for row in csv.DictReader(f):
            if CONV_RE.search(row["Kernel_Name"]):
                rows.append((int(row["Dispatch_Id"]), int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
    rows.sort()
    nf = len(rows) // per_fwd
    fwd = [sum(d for _, d in rows[i * per_fwd:(i + 1) * per_fwd]) / per_fwd / 1e3 for i in range(nf)]
    with open(bench_json) as f:
        b = json.loads([ln for ln in f.read().splitlines() if ln.startswith("{")][-1])
    steps, warm = b["steps"], b["warmup"]
    timed = fwd[warm:warm + steps]
    iso = fwd[warm + steps:warm + steps + 3]  # bench.py's 3 isolated forwards (an ingest pass may follow them)
    rl = b["roofline"]
    res = {"conv_launches_per_forward": per_fwd, "forwards_in_trace": nf,
           "rocprof_avg_us_per_forward_in_launch_order": [round(x, 1) for x in fwd],
           f"rocprof_avg_us_timed_forwards({warm}..{warm + steps - 1})": round(sum(timed) / max(len(timed), 1), 1),
           "rocprof_avg_us_isolated_forwards": round(sum(iso) / max(len(iso), 1), 1),
           "bench_avg_launch_us(events, isolated forwards)": rl["avg_launch_us"],
           "bench_isolated_avg_launch_us": rl.get("isolated_avg_launch_us"),
           "note": "forwards 0..warmup-1 warm-up; then the timed region (two network streams overlapping); "
                   "then the 3 isolated forwards bench.py runs after the timed region (the roofline's timing), then the "
                   "ingest pass if any; B = "
                   f"{b['config']['batch_per_gpu']}"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    return res


def counter_sum(path: str, counter: str):
    tot, n = 0.0, set()
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter or not CONV_RE.search(row.get("Kernel_Name", "")):
                continue
            tot += float(row["Counter_Value"])
            n.add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    return tot, len(n)


def traffic(fetch_csv: str, write_csv: str, key: str, out: str) -> dict:
    fk, nf = counter_sum(fetch_csv, "FETCH_SIZE")
    wk, nw = counter_sum(write_csv, "WRITE_SIZE")
    if nf == 0 or nw == 0:
        raise SystemExit(f"no conv dispatches found ({nf} fetch / {nw} write)")
    fetch_b = 2.0 * fk * 1024 / nf
    write_b = wk * 1024 / nw
    tr = {}
    if os.path.exists(out):
        with open(out) as f:
            tr = json.load(f)
    tr[key] = {"hbm_bytes_per_launch": round(fetch_b + write_b), "fetch_bytes_per_launch": round(fetch_b),
               "write_bytes_per_launch": round(write_b), "conv_dispatches": [nf, nw],
               "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs; KiB -> bytes; "
                         "FETCH_SIZE x2 (gfx950 wide-read correction, MI355X_MICROARCH.md §HBM)"}
    with open(out, "w") as f:
        json.dump(tr, f, indent=1)
    return tr[key]


if __name__ == "__main__":
    if sys.argv[1] == "agree":
        print(json.dumps(agree(*sys.argv[2:5], *(int(a) for a in sys.argv[5:6]))))
    elif sys.argv[1] == "stats":
        print(json.dumps(stats(sys.argv[2], sys.argv[3])["conv_family"]))
    elif sys.argv[1] == "traffic":
        print(json.dumps(traffic(*sys.argv[2:6])))
    else:
        raise SystemExit(__doc__)
