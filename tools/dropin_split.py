#!/usr/bin/env python
"""FrameProcessor.__call__'s stages timed one by one (host perf_counter, medians over --calls frames of the sparse
regime), for the drop-in call's budget:
  stage    = host frame -> pinned buffer (pipeline._pinned)
  h2d      = the async H2D enqueue (+ its device time, from events)
  va_frame = the one C-ABI call: forward + post + grid / A* enqueued, returns after the A* verdict wait
  readback = NavBatch's result copies enqueued + waited for + frame 0 decoded
  paths    = _FrameState + device_paths (Path / Grid objects)
  analyse  = path_analyser
    python tools/dropin_split.py [--calls 300]"""
import argparse
import contextlib
import io
import json
import os
import sys
import time
import warnings

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--pre-streams", type=int, default=0, help="create and use N torch streams first")
    args = ap.parse_args()
    keep = []
    for _ in range(args.pre_streams):
        st_ = torch.cuda.Stream()
        with torch.cuda.stream(st_):
            keep.append(torch.ones(16, device="cuda") * 2)
    torch.cuda.synchronize()
    from bench import regime_kwargs
    from vision_assist_amd import FrameProcessor as fpm
    from vision_assist_amd.FrameProcessor import FrameProcessor
    from vision_assist_amd.post import PLANT_NEVER
    from vision_assist_amd.yolo import YOLO
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        model = YOLO("yolov8s-seg.pt", dtype=args.dtype, **regime_kwargs("sparse", 640)).to("cuda")
    fp = FrameProcessor(model=model, verbose=False, debug=False)
    fp.model = model
    rng = np.random.default_rng(77)
    frames = [rng.integers(0, 256, (640, 640, 3), dtype=np.uint8) for _ in range(16)]
    pipe = fp._pipe(640, 640)
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    per = {}
    T = {k: [] for k in ("stage", "h2d_enqueue", "h2d_device", "va_frame", "readback", "paths", "analyse", "call")}
    with contextlib.redirect_stdout(io.StringIO()):
        for i in range(20 + args.calls):
            f = frames[i % 16]
            t0 = time.perf_counter()
            t = torch.as_tensor(f).reshape(1, 640, 640, 3)
            pinned = pipe._pinned(t)
            t1 = time.perf_counter()
            e0.record(st)
            pipe.load(pinned, st)
            e1.record(st)
            t2 = time.perf_counter()
            batch = pipe.run(None, plant_mode=PLANT_NEVER)
            t3 = time.perf_counter()
            if i >= 20:
                per.setdefault(i % 16, []).append((1e3 * (t3 - t2), batch.rounds))
            fp._adopt(pipe.nav, batch)
            t4 = time.perf_counter()
            paths = fp._state.device_paths() if fp._has_grids() else []
            t5 = time.perf_counter()
            if paths:
                fpm.path_analyser(640, 640, paths)
            t6 = time.perf_counter()
            if i >= 20:
                for k, v in (("stage", t1 - t0), ("h2d_enqueue", t2 - t1), ("va_frame", t3 - t2),
                             ("readback", t4 - t3), ("paths", t5 - t4), ("analyse", t6 - t5), ("call", t6 - t0)):
                    T[k].append(1e3 * v)
                T["h2d_device"].append(e0.elapsed_time(e1))
        # the surface itself, for comparison, and the pieces the split loop does differently
        ts, tin = [], []
        run0 = pipe.run

        def timed_run(*a, **k):
            t = time.perf_counter()
            r = run0(*a, **k)
            tin.append(1e3 * (time.perf_counter() - t))
            return r
        pipe.run = timed_run
        cpu0, wall0 = time.process_time(), time.perf_counter()
        for i in range(args.calls):
            t0 = time.perf_counter()
            fp(frames[i % 16])
            ts.append(1e3 * (time.perf_counter() - t0))
        cpu_ratio = (time.process_time() - cpu0) / (time.perf_counter() - wall0)
        pipe.run = run0
        # the same calls paced by a 1 ms sleep: a stall every N calls or every T ms?
        tsl = []
        for i in range(args.calls):
            time.sleep(0.001)
            t0 = time.perf_counter()
            fp(frames[i % 16])
            tsl.append((t0, 1e3 * (time.perf_counter() - t0)))
        # the surface's body step by step (FrameProcessor.__call__, debug off)
        from vision_assist_amd import _lib
        R = {k: [] for k in ("as_tensor+pipe", "load", "va_frame", "adopt", "checks", "device_paths", "analyser")}
        for i in range(args.calls):
            frame = frames[i % 16]
            c0 = time.perf_counter()
            fp.frame = frame
            t = torch.as_tensor(frame)
            H, W = int(t.shape[0]), int(t.shape[1])
            p_ = fp._pipe(H, W)
            c1 = time.perf_counter()
            p_.load(t.reshape(1, H, W, 3))
            c1b = time.perf_counter()
            b = p_.run(None, plant_mode=PLANT_NEVER)
            c2 = time.perf_counter()
            fp._adopt(p_.nav, b)
            c3 = time.perf_counter()
            if not fp._has_grids():
                continue
            st_ = fp._state
            st_.penalties_assigned = True
            if not st_.nf.peaks:
                print("No protrusions detected.")
            for q in st_.nf.queries:
                if q["status"] != _lib.VA_QUERY_FOUND:
                    print("No path found.")
            c4 = time.perf_counter()
            paths_ = st_.device_paths()
            c5 = time.perf_counter()
            fpm.path_analyser(H, W, paths_)
            c6 = time.perf_counter()
            for k, a_, b_ in (("as_tensor+pipe", c0, c1), ("load", c1, c1b), ("va_frame", c1b, c2), ("adopt", c2, c3), ("checks", c3, c4),
                              ("device_paths", c4, c5), ("analyser", c5, c6)):
                R[k].append(1e3 * (b_ - a_))
        tin = np.array(tin)
        rest = np.array(ts) - tin
        import gc
        gc.collect()
        gc.disable()
        tg = []
        for i in range(args.calls):
            t0 = time.perf_counter()
            fp(frames[i % 16])
            tg.append(1e3 * (time.perf_counter() - t0))
        gc.enable()
        tp, tr = [], []
        for i in range(args.calls):
            t = torch.as_tensor(frames[i % 16]).reshape(1, 640, 640, 3)
            t0 = time.perf_counter()
            t.is_pinned()
            tp.append(1e3 * (time.perf_counter() - t0))
            t0 = time.perf_counter()
            b = pipe.run(t, plant_mode=PLANT_NEVER)
            b.frame(0)
            tr.append(1e3 * (time.perf_counter() - t0))
    out = {k: round(float(np.median(v)), 4) for k, v in T.items()}
    out["va_frame_by_frame"] = {k: [round(float(np.median([x for x, _ in v])), 3), sorted({r for _, r in v})]
                                for k, v in sorted(per.items())}
    out["surface_call_median_ms"] = round(float(np.median(ts)), 4)
    out["surface_calls_per_s"] = round(1e3 / float(np.mean(ts)), 1)
    out["surface_pct_ms"] = {q: round(float(np.percentile(ts, q)), 3) for q in (10, 50, 90, 99)}
    out["surface_max_ms"] = round(float(np.max(ts)), 3)
    out["surface_run_pct_ms"] = {q: round(float(np.percentile(tin, q)), 3) for q in (10, 50, 90, 99, 100)}
    out["surface_host_rest_pct_ms"] = {q: round(float(np.percentile(rest, q)), 3) for q in (10, 50, 90, 99, 100)}
    out["replica_pct_ms"] = {k: [round(float(np.percentile(v, q)), 3) for q in (50, 90, 99, 100)] for k, v in R.items()}
    out["env_ROC_ACTIVE_WAIT_TIMEOUT"] = os.environ.get("ROC_ACTIVE_WAIT_TIMEOUT")
    out["surface_process_cpu_per_wall"] = round(cpu_ratio, 3)
    try:  # per-thread CPU ticks, busiest first: (name, utime + stime)
        import glob as _g
        th = []
        for d in _g.glob("/proc/self/task/*"):
            name = open(d + "/comm").read().strip()
            f = open(d + "/stat").read().rsplit(")", 1)[1].split()
            th.append((name, int(f[11]) + int(f[12])))
        out["thread_ticks"] = sorted(th, key=lambda x: -x[1])[:20]
    except OSError:
        pass
    try:
        out["threads"] = int([l for l in open("/proc/self/status") if l.startswith("Threads")][0].split()[1])
    except OSError:
        pass
    slow = [(round(1e3 * (t - tsl[0][0]), 1), round(d, 2)) for t, d in tsl if d > 5]
    out["paced_slow_calls_at_ms"] = slow[:20]
    out["surface_slowest"] = [(int(i), round(float(ts[i]), 3)) for i in np.argsort(ts)[-8:]]
    out["surface_gc_off_calls_per_s"] = round(1e3 / float(np.mean(tg)), 1)
    out["surface_gc_off_pct_ms"] = {q: round(float(np.percentile(tg, q)), 3) for q in (50, 90, 99)}
    out["is_pinned_pageable_ms"] = round(float(np.median(tp)), 4)
    out["pipe_run_pageable_plus_frame0_ms"] = round(float(np.median(tr)), 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
