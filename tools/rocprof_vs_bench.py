"""rocprofv3 kernel trace of `bench.py --extras none` vs the bench line's own HIP-event timing of the dominant
kernel family (the conv-family launches of the isolated forwards bench.py times after its timed region).
python tools/rocprof_vs_bench.py TRACE.csv BENCH.json [launches_per_forward [warmup steps]] -> JSON on stdout.
The trace's forwards in launch order: warmup, steps timed ones, the 3 isolated ones bench.py times after the timed
region, then the ingest pass's (warm-up + steps) if the run had one."""
import csv
import json
import sys


def is_conv(name: str) -> bool:
    return ("conv" in name or "pw_kernel" in name or "c2f" in name or "stem" in name) and "sppf" not in name


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    per = int(sys.argv[3]) if len(sys.argv) > 3 else 62
    warm = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 10
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    conv = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if is_conv(r["Kernel_Name"])]
    nf = len(conv) // per
    fw = [sum(conv[i * per:(i + 1) * per]) / per / 1000.0 for i in range(nf)]
    line = next(json.loads(l) for l in open(bench) if l.startswith('{"metric'))
    rl = line.get("roofline") or {}
    out = {"conv_launches_per_forward": per, "forwards_in_trace": nf,
           "rocprof_avg_us_per_forward_in_launch_order": [round(v, 1) for v in fw],
           "rocprof_avg_us_timed_forwards": round(sum(fw[warm:warm + steps]) / steps, 1) if nf >= warm + steps else None,
           "rocprof_avg_us_isolated_forwards": (round(sum(fw[warm + steps:warm + steps + 3]) / 3, 1)
                                                if nf >= warm + steps + 3 else None),
           "bench_avg_launch_us(events, isolated forwards)": rl.get("avg_launch_us"),
           "note": "forwards 0..warmup-1 warm-up, then the timed region (two network streams overlapping), then the "
                   "3 isolated forwards bench.py times after the timed region (the roofline's timing), then the ingest pass's"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
