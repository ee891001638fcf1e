#!/usr/bin/env python
"""Per-layer PMC summary of tools/pmc_forward.py runs under rocprofv3 (CPU side; commit the output).

  pmc_summary.py <plan.json> <out.json> <counter_collection.csv> [more csv ...]

The dispatches of our library (kernel names containing '_kernel' inside the anonymous namespace) are taken in
dispatch order; the last forward's n (= ops of the plan) are mapped to the plan's op names.  Per op: the raw
counters, plus
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES x 4 SIMDs ... see note)  [as a fraction]
  wait_frac   = SQ_WAIT_ANY / SQ_WAVE_CYCLES        (waves parked on s_waitcnt / barrier)
  stall_frac  = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (issue stalls)
  hbm_bytes   = 2 x FETCH_SIZE KiB x 1024 + WRITE_SIZE KiB x 1024 (MI355X_MICROARCH.md §HBM gfx950 correction)
  clock_ghz   = GRBM_GUI_ACTIVE / 8 / kernel duration
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

SIMDS = 4 * 256  # SQ_BUSY_CYCLES is summed over the SEs/XCDs; MFMA busy is summed over the SIMDs (see note)


def load(paths):
    disp = defaultdict(dict)  # dispatch id -> {counter: value, _name, _dur}
    for p in paths:
        for f in glob.glob(p):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    d = disp[int(row["Dispatch_Id"])]
                    d["_name"] = row["Kernel_Name"]
                    d["_dur_ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                    d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    return disp


def main():
    plan_path, out_path, csvs = sys.argv[1], sys.argv[2], sys.argv[3:]
    with open(plan_path) as f:
        plan = json.load(f)
    ops = plan["ops"]
    n = len(ops)
    rows_by_pass = []
    for c in csvs:
        disp = load([c])
        ours0 = [disp[k] | {"_id": k} for k in sorted(disp) if "_kernel" in disp[k]["_name"] and ("anonymous" in disp[k]["_name"] or "_GLOBAL__N_" in disp[k]["_name"])]
        # a split-K conv is two dispatches (the slices, then conv2_reduce_kernel): the reduce's counters and time are
        # added to its conv's, one row per op
        ours = []
        for d in ours0:
            if "conv2_reduce_kernel" in d["_name"] and ours:
                prev = ours[-1]
                for k, v in d.items():
                    if not k.startswith("_"):
                        prev[k] = prev.get(k, 0.0) + v
                prev["_dur_ns"] += d["_dur_ns"]
            else:
                ours.append(dict(d))
        if len(ours) < n:
            raise SystemExit(f"{c}: {len(ours)} library dispatches < {n} ops")
        rows_by_pass.append(ours[-n:])  # the last forward
    out = []
    for i, op in enumerate(ops):
        km = re.search(r"(\w+_kernel(<[^()]*>)?)", rows_by_pass[0][i]["_name"])
        r = {"i": i, "name": op["name"], "kernel": (km.group(1) if km else rows_by_pass[0][i]["_name"])[:80]}
        for rows in rows_by_pass:
            for k, v in rows[i].items():
                if not k.startswith("_"):
                    r[k] = v
            r["dur_us"] = round(rows[i]["_dur_ns"] / 1e3, 2)
        wc = r.get("SQ_WAVE_CYCLES")
        if wc:
            if "SQ_WAIT_ANY" in r:
                r["wait_frac"] = round(r["SQ_WAIT_ANY"] / wc, 3)
            if "SQ_WAIT_INST_ANY" in r:
                r["stall_frac"] = round(r["SQ_WAIT_INST_ANY"] / wc, 3)
            if "SQ_ACTIVE_INST_ANY" in r:
                r["active_frac"] = round(r["SQ_ACTIVE_INST_ANY"] / wc, 3)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in r and "GRBM_GUI_ACTIVE" in r and r["GRBM_GUI_ACTIVE"]:
            # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles: per-XCD kernel cycles = /8; MFMA busy is summed over
            # the 256 CUs' 4 SIMDs (32 SIMDs per XCD x 8) -> fraction of the SIMD-cycles the kernel spanned
            r["mfma_busy"] = round(r["SQ_VALU_MFMA_BUSY_CYCLES"] / (r["GRBM_GUI_ACTIVE"] / 8 * SIMDS), 4)
            r["clock_ghz"] = round(r["GRBM_GUI_ACTIVE"] / 8 / (r["dur_us"] * 1e3), 3)
        if "TCP_TCC_READ_REQ_sum" in r:
            r["l1_l2_read_req"] = r["TCP_TCC_READ_REQ_sum"]  # vL1D -> L2 read requests (one per missed line)
        if "FETCH_SIZE" in r or "WRITE_SIZE" in r:
            r["hbm_bytes"] = round(2 * r.get("FETCH_SIZE", 0) * 1024 + r.get("WRITE_SIZE", 0) * 1024)
        if op.get("flops") and r.get("GRBM_GUI_ACTIVE"):
            # the same fraction predicted from the op's FLOPs: f32 16x16x4 = 64, bf16 = 1024 FLOP / cycle / SIMD
            fpc = 64.0 if plan["dtype"] == "f32" else 1024.0
            r["mfma_busy_from_flops"] = round(op["flops"] / fpc / (r["GRBM_GUI_ACTIVE"] / 8 * SIMDS), 4)
        if op.get("flops") and r.get("dur_us"):
            r["tflops"] = round(op["flops"] / (r["dur_us"] * 1e-6) / 1e12, 1)
        out.append(r)
    res = {"plan": {k: plan[k] for k in ("dtype", "scale", "res", "batch")}, "sources": csvs,
           "note": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs); SQ_VALU_MFMA_BUSY_CYCLES "
                   "counts cycles (MI355X_MICROARCH.md); wait/stall/active fractions of SQ_WAVE_CYCLES",
           "ops": out}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    for r in out:
        print(json.dumps({k: r.get(k) for k in ("i", "name", "dur_us", "tflops", "mfma_busy", "wait_frac", "stall_frac",
                                                  "hbm_bytes", "clock_ghz", "l1_l2_read_req") if k in r}))


if __name__ == "__main__":
    main()
