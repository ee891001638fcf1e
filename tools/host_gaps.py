"""Host scheduling gaps: spin on perf_counter for --secs seconds and list every gap longer than --min-ms between
two consecutive reads (a descheduled or stalled thread), with the gaps' spacing.  --gpu: after initialising HIP
through torch (one device allocation), to compare.  Diagnostic only."""
import argparse
import json
import time

ap = argparse.ArgumentParser()
ap.add_argument("--secs", type=float, default=2.0)
ap.add_argument("--min-ms", type=float, default=1.0)
ap.add_argument("--gpu", action="store_true")
a = ap.parse_args()
if a.gpu:
    import torch
    x = torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
gaps = []
t_end = time.perf_counter() + a.secs
last = time.perf_counter()
t0 = last
while last < t_end:
    t = time.perf_counter()
    if t - last > a.min_ms * 1e-3:
        gaps.append((round(1e3 * (last - t0), 2), round(1e3 * (t - last), 3)))
    last = t
starts = [g[0] for g in gaps]
print(json.dumps({"gpu": a.gpu, "secs": a.secs, "n_gaps": len(gaps), "gaps_ms": gaps[:40],
                  "spacing_ms": [round(b - x, 1) for x, b in zip(starts, starts[1:])][:40],
                  "total_gap_ms": round(sum(g[1] for g in gaps), 2)}))
