#!/usr/bin/env python
"""Per-stage CPU time of the REFERENCE's grid path next to the oracle restatement bench.py times as its
cpu_baseline (this container only: it imports /root/reference through the SURVEY.md Appendix C recipe of
tests/golden/gen_goldens.py -- cv2 / ultralytics stubs, cv2 results handed over at the post-cv2 boundary).

Workload = SURVEY.md §6 S1: the 13 reference fixtures resampled to 640x640 (32 x 32 cells), REPS passes in
one process state, median per stage.  Run on one core:
    taskset -c 0 python tools/cpu_stage_compare.py --json profiles/r02/cpu_stage_compare.json
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import statistics
import sys
import tempfile
import time
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    import gen_goldens as G
    from oracle import nav as onav
    from vision_assist_amd.models import Grid, Path
    from vision_assist_amd.PathAnalyser import PathAnalyser
    from workloads.corridors import cells_rect, cells_to_mask, fixture_640

    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    G._install_stubs(tempfile.mkdtemp(prefix="va_oracle_"))
    runner = G.RefRunner()
    fixtures = [fixture_640(g) for _, g in sorted(G.load_fixtures().items())]
    fp, PA = runner.fp, runner.PA
    clk = time.perf_counter
    ref_t = {k: [] for k in ("grid", "penalty", "graph", "protrusion", "astar+paths", "analyser")}
    orc_t = {k: [] for k in ("grid", "penalty", "graph", "protrusion", "astar+paths", "path+analyser")}
    runner.reset_process_state()
    pf = onav.PathFinderOracle()
    analyser = PathAnalyser(clock=lambda: 1_000_000.0)
    quiet = contextlib.redirect_stdout(io.StringIO())
    with quiet:
        for _ in range(args.reps):
            for g in fixtures:
                H, W = 20 * g.shape[0], 20 * g.shape[1]
                # reference (FrameProcessor.__call__ :325-349, stage by stage)
                fp.frame = np.zeros((H, W, 3), dtype=np.uint8)
                G._Harness.mask, G._Harness.rect = cells_to_mask(g), cells_rect(g)
                res = types.SimpleNamespace(masks=types.SimpleNamespace(
                    xy=[np.array([[0, 0], [1, 0], [1, 1]], dtype=np.float32)]))
                t0 = clk()
                fp._extract_grid_information([res])
                t1 = clk()
                fp._calculate_penalties()
                t2 = clk()
                graph = fp._create_graph()
                t3 = clk()
                peaks = fp.protrusion_detector(fp.frame, fp.grids, fp.grid_lookup)
                t4 = clk()
                paths = fp._find_paths(peaks, graph)
                t5 = clk()
                PA.path_analyser(H, W, paths)
                t6 = clk()
                for k, a, b in (("grid", t0, t1), ("penalty", t1, t2), ("graph", t2, t3), ("protrusion", t3, t4),
                                ("astar+paths", t4, t5), ("analyser", t5, t6)):
                    ref_t[k].append(b - a)
                # oracle restatement, as bench.py's cpu_baseline runs it
                st = {}
                nav = onav.frame_nav(cells_to_mask(g), cells_rect(g), H, W, pf, timings=st)
                hits = [q for q in nav["queries"] if q[2]]
                found = [([Grid(**c.model_dump()) for c in q[2]], q[3]) for q in hits]
                tp = clk()
                ps = [Path(grids=cells, total_cost=float(cost), path_type="path") for cells, cost in found]
                by_list = {id(q[2]): p for q, p in zip(hits, ps)}
                analyser(H, W, [by_list[id(c)] for c, _ in nav["paths"]])
                st["path+analyser"] = clk() - tp
                for k in orc_t:
                    orc_t[k].append(st.get(k, 0.0))

    def summ(t):
        med = {k: round(1e3 * statistics.median(v), 3) for k, v in t.items()}
        mean = {k: round(1e3 * statistics.fmean(v), 3) for k, v in t.items()}
        return {"median_ms": med, "mean_ms": mean, "total_median_ms": round(sum(med.values()), 3),
                "total_mean_ms": round(sum(mean.values()), 3)}

    out = {"workload": f"13 reference fixtures resampled to 640x640 (32x32 cells), {args.reps} passes, one process "
                       "state (warm angle cache), per-frame stage times",
           "cores": len(os.sched_getaffinity(0)),
           "reference": summ(ref_t), "oracle_restatement": summ(orc_t),
           "note": "reference = /root/reference code itself (cv2 stubbed at the post-cv2 boundary, as in "
                   "tests/golden/gen_goldens.py); its Path(...) sections/corners run inside _find_paths"}
    print(json.dumps(out, indent=1))
    if args.json:
        os.makedirs(os.path.dirname(args.json), exist_ok=True)
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
