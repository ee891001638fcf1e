"""Single-frame latency (BASELINE.json configs[1], C2: YOLOv8n-seg 640x640 on 1 MI355X; exact f32 by default,
the reference's precision): one frame resident in HBM -> segmentation forward (+ post-processing +
grid/penalty/protrusion/A* for `end_to_end`), synchronised after every frame; median and p90 over --iters runs
after a warm-up, planted corridor masks so the nav stage always runs.  `*_graph`: the frame copy, network and
post-processing replayed as one captured HIP graph.  Prints one JSON line.
    python tools/latency.py [--scale n] [--res 640] [--iters 200] [--dtype f32|bf16]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", default="n")
    ap.add_argument("--res", type=int, default=640)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--graph", action="store_true", help="also time the captured-graph variants")
    args = ap.parse_args()
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_ALWAYS
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    from workloads.corridors import cells_rect, corridor_cells
    H = W = args.res
    arch = Arch(args.scale)
    pipe = FramePipeline(arch, fold(arch, synthetic_state_dict(arch, seed=0)), 1, H, W, dtype=args.dtype)
    g = corridor_cells(11, H // 20, W // 20)
    pc = torch.tensor(g[None].astype(np.uint8)).cuda()
    pr = torch.tensor(np.array([cells_rect(g)], dtype=np.int32)).cuda()
    frame = torch.randint(0, 256, (1, H, W, 3), generator=torch.Generator().manual_seed(1), dtype=torch.uint8).cuda()
    out = {"config": f"C2 shape: YOLOv8{args.scale}-seg {H}x{W} {args.dtype}, batch 1, 1 MI355X", "iters": args.iters}
    variants = [("seg_only", lambda: pipe.run_seg_only()),
                ("end_to_end", lambda: pipe.run(frame, pc, pr, PLANT_ALWAYS))]
    # every variant runs on a stream of its own (graph replays are on SegPostGraph's private stream, ordered after
    # and before this one by events)
    run_stream = torch.cuda.Stream()
    if args.graph:
        # the frame copy + network + post-processing captured once as a HIP graph (the nav stage reads a device
        # flag on the host per speculative A* round, so it stays eager)
        from vision_assist_amd.pipeline import SegPostGraph
        graph = SegPostGraph(pipe, frame, pc, pr, PLANT_ALWAYS, warmup=3)

        def graph_e2e():
            graph.replay()
            pipe.nav_run()

        variants += [("seg_post_graph", graph.replay), ("end_to_end_graph", graph_e2e)]
    for name, fn in variants:
        print(name, file=sys.stderr, flush=True)
        run_stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(run_stream):
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.iters):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
        ts = np.array(ts) * 1e3
        out["ndet"] = int(pipe.post.ndet[0])
        out[name] = {"median_ms": round(float(np.median(ts)), 3), "p90_ms": round(float(np.percentile(ts, 90)), 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
