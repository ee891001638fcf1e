"""C2 end-to-end path alone (bench.c2_latency's pipeline: n-seg 640 bf16, batch 1, the sparse regime's network
masks), for a kernel trace:  rocprofv3 --kernel-trace --stats -d gpurun_out/c2 -- python tools/c2_prof.py
Prints the wall-clock median per frame; the trace gives each kernel's share and the GPU idle gaps."""
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
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--regime", default="sparse")
    ap.add_argument("--lanes", type=int, default=1)
    ap.add_argument("--seg-only", action="store_true", help="bench.c2_latency's seg_only leg (run_seg_only) instead")
    ap.add_argument("--scale", default="n")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--dtype", default="bf16", help="bf16 (C2) or f32 (the drop-in's batch-1 network)")
    a = ap.parse_args()
    if a.batch > 1 and not a.seg_only:
        raise SystemExit("--batch > 1 only with --seg-only")
    import bench
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_IF_NONE
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    from workloads.corridors import cells_rect, corridor_cells
    dev = torch.device("cuda", 0)
    arch = Arch(a.scale)
    pipe = FramePipeline(arch, fold(arch, synthetic_state_dict(arch, seed=0, **bench.regime_kwargs(a.regime, 640))),
                         a.batch, 640, 640, dtype=a.dtype, device=dev, lanes=bool(a.lanes))
    g = corridor_cells(11, 32, 32)
    pc = torch.tensor(g[None].astype(np.uint8), device=dev)
    pr = torch.tensor(np.array([cells_rect(g)], dtype=np.int32), device=dev)
    frame = torch.randint(0, 256, (1, 640, 640, 3), generator=torch.Generator().manual_seed(1),
                          dtype=torch.uint8).to(dev)
    st = torch.cuda.Stream(device=dev)
    st.wait_stream(torch.cuda.current_stream())
    ts = []
    with torch.cuda.stream(st):
        for i in range(20 + a.iters):
            t0 = time.perf_counter()
            if a.seg_only:
                pipe.run_seg_only(stream=st)
            else:
                pipe.run(frame, pc, pr, PLANT_IF_NONE, stream=st)
            st.synchronize()
            if i >= 20:
                ts.append(time.perf_counter() - t0)
    ts = np.array(ts) * 1e3
    key = "seg_only_median_ms" if a.seg_only else "end_to_end_median_ms"
    print(json.dumps({key: round(float(np.median(ts)), 4), "iters": a.iters,
                      "ndet": int(pipe.post.ndet[0]), "lanes": a.lanes}))


if __name__ == "__main__":
    main()
