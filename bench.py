#!/usr/bin/env python
"""bench.py -- frames/s end-to-end (seg + mask + grid + penalty + protrusion + A*) at 640x640 on MI355X.

Workload (BASELINE.json configs[2], "C3"): YOLOv8s-seg, 640x640 frames, post-processing,
grid/penalty/protrusion/A* on the GPU.  The headline runs the network at f32 precision -- the
reference's (model/runs/segment/train16/args.yaml:43 `half: false`, north_star "logits within
1e-3 fp32"): every f32 operand is split exactly into three bf16 terms and the six leading term
products run on the bf16 MFMA (exact products, f32 accumulation; va_seg.hip conv2_kernel SPL,
VA_F32_SPLIT=0 selects the f32 MFMA `v_mfma_f32_16x16x4_f32` instead).  The bf16 MFMA pipeline is
measured in the same run and reported under "bf16".

One step = one pass of the fused hot path (vision_assist_amd.pipeline) over one batch of
--batch synthetic frames per GPU (uint8 BGR, resident in HBM before the timed region;
random-init weights of the yolov8s-seg architecture -- no checkpoints exist offline).
Navigation runs on the network's mask when it yields one and on a planted mask otherwise
(13 reference fixtures resampled to 640x640 + seeded procedural corridors); the
default "sparse" regime gives 1-5 compact detections per frame (a trained model's frames), so
the network's own masks reach the mask choice, contours and A* -- the "dense" / "dense_box"
extras (300 detections per frame) are the post-processing-heavy counterparts.

Multi-GPU: one process per GPU, frames sharded, no collective on the data path; a gloo (CPU)
process group only for the barrier + max-over-ranks timing.  `bench.py --gpus N` starts its N
rank processes itself (before any GPU call) when it is not already running under a launcher;
under torch.distributed.run (the driver's form) it checks WORLD_SIZE == --gpus.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import ctypes
import gc
import gzip
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# dense MFMA peaks, MI355X_MICROARCH.md chip table (fp8: the block-scaled e4m3 MFMA the fp8 convs run on)
# (w8a16: e4m3 weight bytes converted to bf16 in the bf16 kernels' A stage, the bf16 MFMA)
PEAK_TFLOPS = {"bf16": 2500.0, "f32": 157.3, "fp8": 5000.0, "w8a16": 2500.0}
# per-GPU batch (sweeps: DESIGN.md §5; fp8 / w8a16: C5's 64 / 8 GPUs)
DEFAULT_BATCH = {"f32": 256, "bf16": 384, "fp8": 8, "w8a16": 8}
PROF_KINDS = 8
C5_REGIME = "dense_box"  # the regime extras.c5 runs in: the one its chain-parity tests cover
# C5's kept form (the faster form that reaches chain agreement >= 0.75 in dense_box): w8a16 (e4m3
# weights, bf16 activations) at chosen 0.75 / cells 0.875 / paths 0.875; w8a8 (e4m3 MFMA) at 0.25 / 0.75 / 0.75
C5_FORM = "w8a16"


def f32_split_terms() -> int:
    """bf16 term products per f32 product in the f32 convs (va_seg.hip f32_split(): VA_F32_SPLIT, default 6)."""
    e = os.environ.get("VA_F32_SPLIT")
    if e is None:
        return 6
    return 9 if e.startswith("9") else 6 if e.startswith("6") else 0
CONV_KINDS = (1, 5, 6, 7)  # va355.h VA_OP_CONV, VA_OP_CONV0, VA_OP_C2F, VA_OP_STEM


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--dtype", default="f32", choices=["f32", "bf16", "fp8", "w8a16"],
                   help="network arithmetic of the headline (fp8: the convs on e4m3 MFMA, BASELINE configs[4]; "
                        "w8a16: e4m3 weight bytes converted in the bf16 kernels, bf16 activations and MFMA)")
    p.add_argument("--batch", type=int, default=0, help="frames per step per GPU (0 = the dtype's default)")
    p.add_argument("--scale", default="s")
    p.add_argument("--res", type=int, default=640)
    p.add_argument("--regime", default="sparse", choices=["sparse", "natural", "mid", "dense", "dense_box"],
                   help="detection regime of the synthetic weights (regime_kwargs); the headline is 'sparse': 1-5 "
                        "compact detections per frame through decode / NMS / contours / mask choice, planted "
                        "navigation masks only on frames without a detection")
    p.add_argument("--extras", default="c4,c2,dropin,dealer,bf16,dense,dense_box,c5,c5_w8a8",
                   help="comma list of extra measurements in the same run: c4 (BASELINE configs[3]: one frame per GPU "
                        "per step, s-seg f32), c2 (configs[1]: n-seg bf16 batch-1 latency, seg-only and end to end), "
                        "dropin (FrameProcessor.__call__ per frame from host numpy frames, answers included), "
                        "dealer (one frame source dealt to a FrameProcessor worker process per GPU, in-order answers), "
                        "bf16 (the bf16 MFMA pipeline), "
                        "dense (300 detections per frame, the random weights' noise masks), dense_box (300 "
                        "detections per frame with solid box masks, one contour each, as a trained model's compact "
                        "masks), c5 (YOLOv8m-seg 1280, batch 8, C5's kept form: e4m3 weight bytes converted to bf16 in "
                        "the kernels, bf16 activations), c5_w8a8 (the same on the e4m3 MFMA with e4m3 activations); 'none' to skip")
    p.add_argument("--cpu-sample", type=int, default=256,
                   help="frames timed for the CPU baseline (0 = skip; 256 = ~10-20 s)")
    p.add_argument("--no-prof", action="store_true", help="skip the HIP-event timing of the isolated forwards")
    p.add_argument("--no-ingest", action="store_true",
                   help="skip the PCIe-inclusive pass (frames from pinned host memory; reported as `ingest`)")
    p.add_argument("--no-overlap", action="store_true",
                   help="serial steps (no overlap of batch k's grid stage with batch k+1's network)")
    p.add_argument("--pipelines", type=int, default=3,
                   help="batches in flight (buffer sets): 3 lets batch k+2's network be enqueued before the "
                        "host blocks in batch k's grid stage")
    p.add_argument("--seg-streams", type=int, default=2, choices=[1, 2, 3, 4],
                   help="network streams of the overlapped pipeline (2: consecutive forwards run concurrently)")
    p.add_argument("--c4-pipelines", type=int, default=6,
                   help="frames in flight per GPU in the c4 extra (batch 1: more concurrent forwards fill the chip)")
    p.add_argument("--c4-seg-streams", type=int, default=3, choices=[1, 2, 3, 4],
                   help="network streams of the c4 extra (3 + the grid stage's stream: one hardware queue each)")
    # dealer defaults from the round-5 sweep (profiles/r05/dealer/): 2 workers x 16 frames x 128 slots 3,858-4,031
    # frames/s per GPU; 1 x 32 x 64 2,670; 3 x 16 3,984; 4 x 16 3,637; 2 x 8 3,341
    p.add_argument("--dealer-workers-per-gpu", type=int, default=2,
                   help="FrameProcessor worker processes per GPU in the dealer extra (each its own PathFinder shard)")
    p.add_argument("--dealer-batch", type=int, default=16,
                   help="frames a dealer worker runs as one device batch (up to; what waits in its ring)")
    p.add_argument("--dealer-slots", type=int, default=128, help="ring slots per dealer worker")
    p.add_argument("--dealer-readers", type=int, default=0,
                   help="reader threads copying frames into the dealer's rings (0: the calling thread)")
    p.add_argument("--dropin-only", action="store_true",
                   help="print only the dropin measurement's JSON (the dropin extra runs this in a child process)")
    return p.parse_args()


def regime_kwargs(regime: str, res: int) -> dict:
    """synthetic_state_dict keywords of a detection regime: 'sparse' = one live class whose bias
    leaves ~1-5 detections per frame with solid (compact) masks, as a trained model's frames; 'natural' =
    Ultralytics' prior bias (no detections on noise frames: A* runs on planted masks); 'mid' = bias 0 (saturates
    max_det on these weights); 'dense' = +4 (300 noise masks); 'dense_box' = +4 with solid box masks."""
    return {"sparse": {"sparse": res}, "natural": {}, "mid": {"cls_bias": 0.0}, "dense": {"cls_bias": 4.0},
            "dense_box": {"cls_bias": 4.0, "solid_masks": True}}[regime]


def planted_pool(n: int, res: int, seed: int):
    """Planted navigation masks: the reference's 13 fixtures (from the committed goldens) resampled to
    the frame + seeded procedural corridors."""
    from workloads.corridors import cells_rect, corridor_cells, fixture_640
    R = C = res // 20
    grids = []
    path = os.path.join(REPO, "tests", "golden", "nav_goldens.json.gz")
    if res == 640 and os.path.exists(path):
        with gzip.open(path, "rt") as f:
            fx = json.load(f)["fixtures"]
        for name in sorted(fx):
            g = np.array([[ch == "1" for ch in row] for row in fx[name]], dtype=bool)
            grids.append(fixture_640(g))
    i = 0
    while len(grids) < n:
        grids.append(corridor_cells(seed * 7919 + i, R, C))
        i += 1
    grids = grids[:n]
    rng = np.random.default_rng(seed)
    rng.shuffle(grids)
    cells = np.stack(grids).astype(np.uint8)
    rects = np.array([cells_rect(g) for g in grids], dtype=np.int32)
    return cells, rects


def cpu_baseline(arch, fw, frames_u8: np.ndarray, plant_cells, plant_rects, res: int):
    """The oracle (torch fp32 CPU YOLOv8-seg + post-processing, pure-python grid/A* restatement with the
    reference's algorithmic structure, pydantic Path sections/corners and the analyser) on a bounded
    sample of the same workload.  -> (frames/s, seconds, per-stage ms per frame)."""
    from oracle import nav as onav
    from oracle import yolo_ref as Y
    from vision_assist_amd.models import Grid, Path
    from vision_assist_amd.PathAnalyser import PathAnalyser
    from workloads.corridors import cells_to_mask
    pf = onav.PathFinderOracle()
    analyser = PathAnalyser()
    n = frames_u8.shape[0]
    stages = {}
    t0 = time.perf_counter()
    for i in range(n):
        tn = time.perf_counter()
        with torch.no_grad():
            out = Y.predict(arch, fw, torch.from_numpy(frames_u8[i:i + 1]))
        det, masks = out[0]
        stages["network+post"] = stages.get("network+post", 0.0) + time.perf_counter() - tn
        tm = time.perf_counter()
        # mask -> polygon -> cells: a pure-python findContours / fillPoly port (cv2's C++ is absent), its own lap
        m, rect = Y.select_mask(masks)
        if m is None:  # planted, as on the GPU
            m = cells_to_mask(plant_cells[i].astype(bool))
            rect = tuple(int(v) for v in plant_rects[i])
        else:
            m = m.numpy()
        stages["mask->cells"] = stages.get("mask->cells", 0.0) + time.perf_counter() - tm
        nav = onav.frame_nav(m, rect, res, res, pf, timings=stages)
        # FrameProcessor.py:246 Path(...) (sections + corners) for every found path and :349 path_analyser on
        # the unique ones: the pure-python host classes the product's FrameProcessor surface also runs per
        # frame (the oracle's cells are re-typed as models.Grid outside the timed span)
        hits = [q for q in nav["queries"] if q[2]]
        found = [([Grid(**c.model_dump()) for c in q[2]], q[3]) for q in hits]
        tp = time.perf_counter()
        paths = [Path(grids=cells, total_cost=float(cost), path_type="path") for cells, cost in found]
        if nav["state"].grids:
            by_list = {id(q[2]): p for q, p in zip(hits, paths)}
            analyser(res, res, [by_list[id(cells)] for cells, _ in nav["paths"]])
        stages["path+analyser"] = stages.get("path+analyser", 0.0) + time.perf_counter() - tp
    dt = time.perf_counter() - t0
    per = {k: round(1e3 * v / n, 3) for k, v in stages.items()}
    return n / dt, dt, per


class Run:
    """One measured configuration: pipelines, resident inputs and the timed steps."""

    def __init__(self, args, dev, rank, dtype, B, regime, scale=None, res=None, pipelines=None, seg_streams=None):
        from vision_assist_amd.pipeline import FramePipeline, OverlappedPipelines
        from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
        self.args, self.dtype, self.B, self.regime = args, dtype, B, regime
        self.scale, self.res = scale or args.scale, res or args.res
        self.arch = Arch(self.scale)
        self.fw = fold(self.arch, synthetic_state_dict(self.arch, seed=0, **regime_kwargs(regime, self.res)))
        H = W = self.res
        self.overlap = not args.no_overlap
        if self.overlap:
            self.opipe = OverlappedPipelines(self.arch, self.fw, B, H, W, dtype=dtype, device=dev,
                                             seg_streams=seg_streams or args.seg_streams,
                                             depth=pipelines or args.pipelines)
            self.pipe = self.opipe.a
        else:
            self.pipe = FramePipeline(self.arch, self.fw, B, H, W, dtype=dtype, device=dev)
        # resident inputs: P batches of frames + planted masks, distinct per rank
        self.P = 4
        self.frames, self.pcs, self.prs = [], [], []
        for j in range(self.P):
            rng = np.random.default_rng(1000 * rank + j)
            self.frames.append(torch.from_numpy(rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8)).to(dev))
            c, r = planted_pool(B, self.res, 1000 * rank + j)
            self.pcs.append(torch.from_numpy(c).to(dev))
            self.prs.append(torch.from_numpy(r).to(dev))
        torch.cuda.synchronize()

    def steps(self, n, host=False):
        """n steps; overlapped: batch s+1's network is enqueued before batch s's grid stage runs.  host: the
        frames come from pinned host memory (an H2D copy per batch on its network stream) instead of HBM."""
        from vision_assist_amd.post import PLANT_IF_NONE
        P, rounds, res = self.P, 0, None
        frames = self.hframes if host else self.frames
        if not self.overlap:
            for s in range(n):
                res = self.pipe.run(frames[s % P], self.pcs[s % P], self.prs[s % P], PLANT_IF_NONE)
                rounds += res.rounds
            return rounds, res
        op = self.opipe
        ahead = op.depth - 1
        for s in range(min(ahead, n)):
            op.submit(frames[s % P], self.pcs[s % P], self.prs[s % P], PLANT_IF_NONE)
        for s in range(n):
            if s + ahead < n:
                k = s + ahead
                op.submit(frames[k % P], self.pcs[k % P], self.prs[k % P], PLANT_IF_NONE)
            res = op.finish(s)
            rounds += res.rounds
        return rounds, res

    def ingest(self, steps, world) -> dict:
        """The same steps with the frames in pinned host memory: each batch's uint8 frames cross PCIe (H2D on
        the batch's network stream, overlapped with the other batches in flight) -- the rate a camera-fed
        deployment sees.  Reported beside `value` (which keeps inputs resident in HBM, as the contract asks)."""
        from vision_assist_amd.shard import timed
        self.hframes = [f.cpu().pin_memory() for f in self.frames]
        self.steps(2, host=True)
        torch.cuda.synchronize()
        if self.overlap:
            self.opipe.k = 0
        _, elapsed = timed(lambda: self.steps(steps, host=True), world, sync=torch.cuda.synchronize)
        fps = world * self.B * steps / elapsed
        nbytes = self.res * self.res * 3
        del self.hframes
        return {"pcie_inclusive_value": round(fps, 2), "unit": "frames/s", "h2d_bytes_per_frame": nbytes,
                "h2d_GBps": round(fps * nbytes / world / 1e9, 2),
                "how": "frames in pinned host memory, one H2D copy per batch on its network stream (3 batches in "
                       "flight); all else as the headline"}

    def measure(self, steps, warmup, world, prof=True) -> dict:
        from vision_assist_amd import _lib
        from vision_assist_amd.shard import timed
        args, B, H = self.args, self.B, self.res
        self.steps(warmup)
        torch.cuda.synchronize()
        if self.overlap:
            self.opipe.k = 0
        cpu0, wall0 = time.process_time(), time.perf_counter()
        (rounds, res), elapsed = timed(lambda: self.steps(steps), world, sync=torch.cuda.synchronize)
        host_cpu = (time.process_time() - cpu0) / (time.perf_counter() - wall0)
        res.host()  # (synchronised snapshot of the last batch's records)
        paths = sum(1 for i in range(B) for q in res.frame(i).queries if q["unique"])
        seg = self.pipe.seg
        gflop_alg = seg.gflop_per_frame(H, H)
        gflop_exec = seg.plan_gflop(self.pipe.plan)  # per B-frame forward
        out = {"value": world * B * steps / elapsed, "elapsed": elapsed, "ms_per_step": 1e3 * elapsed / steps,
               "rounds": rounds / steps, "paths": paths, "gflop_alg": gflop_alg, "gflop_exec": gflop_exec,
               "host_cpu": host_cpu}
        if prof:
            out["roofline"] = self.roofline(_lib.load(), gflop_alg, gflop_exec, elapsed, steps)
        return out

    def roofline(self, lib, gflop_alg, gflop_exec, elapsed, steps) -> dict:
        """The conv family's average launch duration, measured with HIP events around every op of 3 forwards
        run ALONE (after the timed region, untimed, on the launch stream): during the timed region two
        forwards share the chip, so an overlapped launch's event span is not that kernel's duration."""
        from vision_assist_amd import _lib
        pipe, B = self.pipe, self.B
        torch.cuda.synchronize()
        nfwd = 3
        _lib.check(lib.va_prof_start(pipe.plan["n"] * nfwd + 16), "va_prof_start")
        for _ in range(nfwd):
            pipe.run_seg_only()
            torch.cuda.synchronize()
        ms, cnt = (ctypes.c_double * PROF_KINDS)(), (ctypes.c_int64 * PROF_KINDS)()
        lib.va_prof_stop(ms, cnt, PROF_KINDS)
        conv_ms, conv_n = sum(ms[k] for k in CONV_KINDS), sum(cnt[k] for k in CONV_KINDS)
        other_ms = sum(ms[k] for k in range(PROF_KINDS) if k not in CONV_KINDS)
        launches = conv_n / nfwd
        fl_exec = gflop_exec * 1e9 / launches
        fl_alg = gflop_alg * B * 1e9 / launches
        avg_s = conv_ms / 1e3 / conv_n
        peak = PEAK_TFLOPS[self.dtype]
        achieved = fl_exec / avg_s / 1e12
        terms = f32_split_terms() if self.dtype == "f32" else 0
        f32eq = None
        if terms:
            # the MFMA the f32 convs execute is bf16 (terms products per f32 product): price the executed bf16
            # MFMA work against the bf16 peak; model.0 is counted once at K = 27 (it runs three term products on
            # the MFMA at K = 32, conv0_f32m, or on the VALU: counting it once under-states, never over-states)
            fl_c0 = sum(m.get("flops_c0", 2.0 * m["M"] * m["N"] * m["K"] if m["name"] == "model.0" else 0.0)
                        for m in pipe.plan["meta"]) / launches
            f32eq = {"achieved": round(achieved, 2), "peak": PEAK_TFLOPS["f32"],
                     "frac": round(achieved / PEAK_TFLOPS["f32"], 5),
                     "def": "f32 GEMM FLOPs per launch / launch time against the f32 MFMA peak (what the exact-f32 "
                            "MFMA form, VA_F32_SPLIT=0, is bounded by)"}
            achieved = (terms * (fl_exec - fl_c0) + fl_c0) / avg_s / 1e12
            peak = PEAK_TFLOPS["bf16"]
        rl = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
              "frac": round(achieved / peak, 5), "traffic": None,
              "kernel": f"the {launches:.0f} conv-family launches of one YOLOv8{self.scale}-seg forward "
                        + (f"(f32 convs on conv3h_kernel's / conv3t_kernel's / conv2_kernel's bf16 three-term forms; "
                           "model.0 on conv0_f32m)" if terms else
                           f"({self.dtype} MFMA GEMM kernels: conv/conv2/conv4/conv_dn/conv_patch/pw/c2f/stem)"),
              "flops_per_launch": round(fl_exec), "flops_per_launch_def": "executed GEMM FLOPs of the plan / launch",
              "avg_launch_us": round(avg_s * 1e6, 3),
              "achieved_algorithmic": round(fl_alg / avg_s / 1e12, 2),
              "flops_per_launch_algorithmic": round(fl_alg),
              "timing": f"HIP events around every op of {nfwd} forwards run alone after the timed region, on the "
                        "launch stream (rocprofv3 kernel trace: profiles/)",
              "forward_ms_isolated": round((conv_ms + other_ms) / nfwd, 3),
              "conv_ms_per_forward_isolated": round(conv_ms / nfwd, 3),
              "step_achieved": round(gflop_exec * steps / elapsed / 1e3, 2),
              "step_achieved_def": "executed conv TFLOP of all timed forwards / timed wall time (per GPU)"}
        if terms:
            rl["f32_equivalent"] = f32eq
            rl["arithmetic"] = (f"f32 operands split exactly into three bf16 terms, {terms} term products per f32 "
                                "product on v_mfma_f32_16x16x32_bf16, f32 accumulation; achieved = executed bf16 MFMA "
                                "FLOPs (terms x f32 GEMM FLOPs) per launch / launch time")
        traffic_file = os.path.join(REPO, "profiles", "conv_traffic.json")
        if os.path.exists(traffic_file):
            with open(traffic_file) as f:
                tr = json.load(f)
            key = f"{self.scale}-{self.res}-b{B}-{self.dtype}"
            if key in tr:
                rl["traffic"] = tr[key]["hbm_bytes_per_launch"]
                rl["traffic_source"] = f"profiles/conv_traffic.json[{key}] (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE)"
        return rl

    def release(self):
        for name in ("opipe", "pipe", "frames", "pcs", "prs"):
            if hasattr(self, name):
                delattr(self, name)
        gc.collect()
        torch.cuda.empty_cache()


def c4_rate(args, dev, rank, world, prof) -> dict:
    """C4 (BASELINE.json configs[3]): YOLOv8s-seg 640x640 f32, ONE frame per GPU per step (batch 8 over 8 GPUs),
    frames dealt round-robin, no collective; the headline's overlapped pipeline with batch 1, --c4-pipelines frames in
    flight per GPU on --c4-seg-streams network streams (6 on 3: 1,031 -> 1,456 frames/s against the headline's 3 on
    2; a 4th network stream shares a hardware queue and fell to 1,015).  value = frames of all ranks /
    max-over-ranks time."""
    steps = max(200, 10 * args.steps)
    r = Run(args, dev, rank, "f32", 1, args.regime, scale="s", res=640, pipelines=args.c4_pipelines,
            seg_streams=args.c4_seg_streams)
    m = r.measure(steps, 20, world, prof)
    r.release()
    e = {"value": round(m["value"], 2), "unit": "frames/s", "ms_per_step": round(m["ms_per_step"], 4), "steps": steps,
         "dtype": "f32", "batch_per_gpu": 1, "global_batch": world, "regime": args.regime,
         "workload": "C4 (BASELINE.json configs[3]): YOLOv8s-seg 640x640, one frame per GPU per step, network masks "
                     f"(planted only when a frame has no detection) -> contours -> grid / A*, {args.c4_pipelines} frames in "
                     f"flight per GPU on {args.c4_seg_streams} network streams",
         "parity": "tests/test_gpu_c4.py (2 ranks, one frame per rank per step, vs the per-shard oracle-chain replay)"}
    if prof:
        rl = m["roofline"]
        e["roofline"] = {k: rl[k] for k in ("achieved", "peak", "frac", "avg_launch_us", "traffic")}
    return e


def c2_latency(args, dev, iters=200) -> dict:
    """C2 (BASELINE.json configs[1]): YOLOv8n-seg 640x640 bf16, batch 1, one frame resident in HBM, synchronised
    after every frame; median / p90 of the seg kernels alone and of the whole path (network masks of the sparse
    regime, a planted corridor when a frame has none), eager launches on a stream of the run's own (the
    graph-replayed form is tools/latency.py --graph: it measured within 1 % of eager)."""
    from vision_assist_amd.pipeline import FramePipeline
    from vision_assist_amd.post import PLANT_IF_NONE
    from vision_assist_amd.seg_arch import Arch, fold, synthetic_state_dict
    from workloads.corridors import cells_rect, corridor_cells
    arch = Arch("n")
    pipe = FramePipeline(arch, fold(arch, synthetic_state_dict(arch, seed=0, **regime_kwargs(args.regime, 640))),
                         1, 640, 640, dtype="bf16", device=dev)
    g = corridor_cells(11, 32, 32)
    pc = torch.tensor(g[None].astype(np.uint8), device=dev)
    pr = torch.tensor(np.array([cells_rect(g)], dtype=np.int32), device=dev)
    frame = torch.randint(0, 256, (1, 640, 640, 3), generator=torch.Generator().manual_seed(1),
                          dtype=torch.uint8).to(dev)
    st = torch.cuda.Stream(device=dev)
    st.wait_stream(torch.cuda.current_stream())

    out = {"workload": "C2 (BASELINE.json configs[1]): YOLOv8n-seg 640x640 bf16, batch 1, 1 MI355X; frame resident "
                       "in HBM, synchronised per frame", "iters": iters, "regime": args.regime}
    for name, fn in (("seg_only", lambda: pipe.run_seg_only(stream=st)),
                     ("end_to_end", lambda: pipe.run(frame, pc, pr, PLANT_IF_NONE, stream=st))):
        with torch.cuda.stream(st):
            for _ in range(20):
                fn()
            st.synchronize()
            ts = []
            for _ in range(iters):
                t0 = time.perf_counter()
                fn()
                st.synchronize()
                ts.append(time.perf_counter() - t0)
        ts = np.array(ts) * 1e3
        out[name] = {"median_ms": round(float(np.median(ts)), 4), "p90_ms": round(float(np.percentile(ts, 90)), 4)}
    out["ndet_last_frame"] = int(pipe.post.ndet[0])
    del pipe
    gc.collect()
    torch.cuda.empty_cache()
    return out


def dropin_rate(args, dev, calls=200) -> dict:
    """The drop-in surface's own rate: main.py:80-82 calls processor(frame) once per frame with a host numpy
    frame.  FrameProcessor.__call__ (YOLO s-seg f32, the sparse regime's network masks) does the H2D copy, one
    batch-1 device pipeline, the host pydantic Path construction (sections, corners) and the PathAnalyser
    answer per call; frames cycle through 16 distinct seeded 640x640 frames."""
    import warnings

    from vision_assist_amd.FrameProcessor import FrameProcessor
    from vision_assist_amd.yolo import YOLO
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        model = YOLO("yolov8s-seg.pt", dtype="f32", **regime_kwargs(args.regime, 640)).to(dev)
    fp = FrameProcessor(model=model, verbose=False, debug=False)
    fp.model = model
    rng = np.random.default_rng(77)
    frames = [rng.integers(0, 256, (640, 640, 3), dtype=np.uint8) for _ in range(16)]
    answers = 0
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):  # "No path found." prints, as the reference's
        for i in range(10):
            fp(frames[i % 16])
        torch.cuda.synchronize()
        c0 = time.process_time()
        t0 = time.perf_counter()
        for i in range(calls):
            a = fp(frames[i % 16])
            answers += a != []
        dt = time.perf_counter() - t0
        host_cpu = (time.process_time() - c0) / dt
    return {"value": round(calls / dt, 2), "unit": "frames/s", "ms_per_call": round(1e3 * dt / calls, 4),
            "calls": calls, "calls_with_answer": answers, "dtype": "f32", "regime": args.regime,
            "host_cpu_per_wall": round(host_cpu, 2),
            "workload": "FrameProcessor.__call__(frame) per frame (main.py:80-82): host numpy 640x640 frame -> pinned "
                        "H2D -> YOLOv8s-seg f32 + post + grid / A* (batch 1) -> host Path sections/corners + "
                        "PathAnalyser answer"}


def dropin_child(args) -> dict:
    """dropin_rate in a fresh child process (`bench.py --dropin-only`): main.py runs FrameProcessor in a process of
    its own, and the streams this bench process has made by then (overlapped pipelines, C4's, C2's) change which
    hardware queues the batch-1 forward's lane streams share -- with three extra streams made first the call took
    1.76 instead of 1.58 ms of device time (profiles/r04/dropin2/streams/)."""
    import subprocess
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--dropin-only", "--regime", args.regime],
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            raise RuntimeError(f"exit status {r.returncode}: {r.stderr[-1500:]}")
        d = json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:  # the headline line is still printed; the extra says what failed
        print(f"dropin child failed: {e}", file=sys.stderr, flush=True)
        return {"value": None, "error": str(e)[-1500:]}
    d["process"] = "a fresh child process (bench.py --dropin-only), as main.py runs FrameProcessor"
    return d


def dealer_rate(args, dev, frames_n: int = 1024) -> dict:
    """SURVEY.md §8e from the drop-in surface: ONE frame source (a reader, as main.py's camera loop) dealing host
    frames round-robin to one FrameProcessor worker process per visible GPU (vision_assist_amd.shard.FrameDealer:
    shared-memory frame ring, in-order answers, each worker with its own PathFinder state), f32 s-seg, the
    regime's network masks.  frames/s of in-order answers over the whole node's workers."""
    from vision_assist_amd.shard import FrameDealer, dropin_worker
    G = max(1, torch.cuda.device_count()) * args.dealer_workers_per_gpu
    ngpu = max(1, torch.cuda.device_count())
    rng = np.random.default_rng(78)
    frames = [rng.integers(0, 256, (640, 640, 3), dtype=np.uint8) for _ in range(16)]
    with FrameDealer(dropin_worker("yolov8s-seg.pt", dtype="f32", batch=args.dealer_batch, quiet=True,
                                   **regime_kwargs(args.regime, 640)),
                     [w % ngpu for w in range(G)], 640, 640, slots=args.dealer_slots,
                     readers=args.dealer_readers) as d:
        for _ in d.map(frames[i % 16] for i in range(32 * G)):  # warm: plans, first launches, lanes' streams
            pass
        t0 = time.perf_counter()
        answers = sum(a != [] for a in d.map(frames[i % 16] for i in range(frames_n)))
        dt = time.perf_counter() - t0
    return {"value": round(frames_n / dt, 2), "unit": "frames/s", "workers": G, "gpus": ngpu, "frames": frames_n,
            "frames_with_answer": answers, "dtype": "f32", "regime": args.regime, "worker_batch": args.dealer_batch,
            "slots": args.dealer_slots, "readers": args.dealer_readers,
            "workload": f"one reader dealing host 640x640 frames round-robin to {args.dealer_workers_per_gpu} "
                        "FrameProcessor worker process(es) per GPU (vision_assist_amd.shard.FrameDealer: shared-memory "
                        "frame ring with shared head / tail counters), answers back in frame order; each worker runs "
                        f"up to {args.dealer_batch} waiting frames as one device batch, two batches in flight "
                        "(pipeline.StreamBatches), answers built frame by frame in order"}


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` (N > 1) started without a torch.distributed.run environment: start N fresh child
    processes of this script, rank r with RANK = LOCAL_RANK = r, WORLD_SIZE = N and a 127.0.0.1 rendezvous, before
    this process has made any GPU call (it never makes one: a process that initialised the GPU must not hand its
    role to another).  Waits for every rank, relays rank 0's JSON line, and returns non-zero if any rank failed
    (the others are then stopped by their exact PIDs)."""
    import socket
    import subprocess
    import tempfile
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out0 = tempfile.TemporaryFile(mode="w+")
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        # rank 0's stdout (the JSON line) to a file, the other ranks' stdout and everyone's stderr to our stderr
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=out0 if r == 0 else sys.stderr, stderr=sys.stderr))
    failed = None
    while failed is None and any(p.poll() is None for p in procs):
        for r, p in enumerate(procs):
            if p.poll() not in (None, 0):
                failed = (r, p.returncode)
                break
        time.sleep(0.2)
    if failed is None:
        failed = next(((r, p.returncode) for r, p in enumerate(procs) if p.returncode != 0), None)
    if failed is not None:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
        print(f"bench.py --gpus {n}: rank {failed[0]} exited with status {failed[1]}", file=sys.stderr, flush=True)
        return failed[1] if failed[1] and failed[1] > 0 else 1
    out0.seek(0)
    lines = [ln for ln in out0.read().splitlines() if ln.startswith("{")]
    if len(lines) != 1:
        print(f"bench.py --gpus {n}: rank 0 printed {len(lines)} JSON lines", file=sys.stderr, flush=True)
        return 1
    print(lines[0], flush=True)
    return 0


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (one rank per GPU)")
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        tdist.init_process_group("gloo")  # barrier + max only: no RCCL communicator on the data path
    # rank r on GPU r of the node (a 1-GPU rehearsal box shares cuda:0 between ranks)
    torch.cuda.set_device(local % torch.cuda.device_count() if dist else 0)
    dev = torch.device("cuda", torch.cuda.current_device())
    if args.dropin_only:
        print(json.dumps(dropin_rate(args, dev)), flush=True)
        return
    B = args.batch or DEFAULT_BATCH[args.dtype]
    prof = not args.no_prof

    run = Run(args, dev, rank, args.dtype, B, args.regime)
    main_res = run.measure(args.steps, args.warmup, world, prof)
    ingest = run.ingest(args.steps, world) if not args.no_ingest else None
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        nsamp = min(args.cpu_sample, run.P * B)
        fr_all = torch.cat(run.frames).cpu().numpy()[:nsamp]
        pc_all = torch.cat(run.pcs).cpu().numpy()[:nsamp]
        pr_all = torch.cat(run.prs).cpu().numpy()[:nsamp]
        arch, fw = run.arch, run.fw
    run.release()
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        ncpu = torch.get_num_threads()
        fps_cpu, dt, per_stage = cpu_baseline(arch, fw, fr_all, pc_all, pr_all, args.res)
        grid_ms = sum(v for k, v in per_stage.items() if k != "network+post")
        # the mask->cells lap is a port-only cost: the reference runs C++ there (ultralytics' masks.xy contours,
        # cv2.contourArea / boundingRect / fillPoly, FrameProcessor.py:72-86), absent from this image, so the
        # oracle's pure-python restatement stands in; the baseline is reported with and without it
        port_ms = per_stage.get("mask->cells", 0.0)
        fps_wo = 1e3 / max(1e3 / fps_cpu - port_ms, 1e-9)
        cpu = {"value": round(fps_cpu, 3), "unit": "frames/s", "cores": ncpu, "kind": "port",
               "value_without_port_only_laps": round(fps_wo, 3),
               "port_only_laps": {"mask->cells": "pure-python findContours/fillPoly port; cv2 C++ in the reference"},
               "grid_stage_ms_per_frame": round(grid_ms, 2),  # pure-python grid ... analyser (1 core)
               "stage_ms_per_frame": per_stage,
               "sample": f"first {nsamp} frames of the resident pool (same frames/masks as the GPU run), {dt:.1f} s: "
                         f"torch fp32 CPU yolov8{args.scale}-seg + decode/NMS/process_mask ({ncpu} threads) + "
                         "pure-python grid/penalty/graph/protrusion/A*/Path sections+corners/analyser restatement "
                         "(oracle/, 1 core)"}

    extras = {}
    for ex in [e for e in args.extras.split(",") if e and e != "none"]:
        if ex == "c2":
            if world == 1:
                extras[ex] = c2_latency(args, dev)
            continue
        if ex == "dropin":
            if world == 1:
                extras[ex] = dropin_child(args)
            continue
        if ex == "dealer":
            if world == 1:
                extras[ex] = dealer_rate(args, dev)
            continue
        if ex == "c4":
            extras[ex] = c4_rate(args, dev, rank, world, prof)
            continue
        if ex == "bf16" and args.dtype != "bf16":
            dt_, B_, reg_ = "bf16", args.batch or DEFAULT_BATCH["bf16"], args.regime
        elif ex in ("dense", "dense_box") and args.regime != ex:
            dt_, B_, reg_ = args.dtype, B, ex
        elif ex == "c5" and not (args.scale == "m" and args.res == 1280 and args.dtype == C5_FORM):
            # C5 runs in the regime its parity tests cover (tests/test_gpu_fp8.py::test_*_chain_1280_vs_fp32_oracle)
            dt_, B_, reg_ = C5_FORM, DEFAULT_BATCH[C5_FORM], C5_REGIME
        elif ex == "c5_w8a8" and not (args.scale == "m" and args.res == 1280 and args.dtype == "fp8"):
            dt_, B_, reg_ = "fp8", DEFAULT_BATCH["fp8"], C5_REGIME
        else:
            continue
        sc_, rs_ = ("m", 1280) if ex in ("c5", "c5_w8a8") else (None, None)
        r = Run(args, dev, rank, dt_, B_, reg_, scale=sc_, res=rs_)
        m = r.measure(args.steps, min(args.warmup, 3), world, prof)
        ing = r.ingest(args.steps, world) if (ex == "bf16" and not args.no_ingest) else None
        r.release()
        e = {"value": round(m["value"], 2), "ms_per_step": round(m["ms_per_step"], 3), "dtype": dt_,
             "batch_per_gpu": B_, "regime": reg_}
        if ex == "c5":
            e["form"] = ("w8a16: every conv's weights (model.0 and the fused 1x1 tails' aside) stored in HBM as e4m3 "
                         "bytes with one f32 scale per output channel (va_conv_args.w8), converted exactly to bf16 in "
                         "the bf16 kernels' A stage, the accumulator scaled in the epilogue; bf16 activations on the "
                         "bf16 MFMA -- kept over the e4m3-MFMA form (c5_w8a8) because only it reaches the chain bar in "
                         "dense_box (DESIGN.md §4.3)")
            e["workload"] = ("C5 (BASELINE.json configs[4]) per GPU: YOLOv8m-seg 1280x1280, e4m3 weights (w8a16), batch "
                             "8 = 64 across 8 GPUs, post-processing + grid / A* on GPU")
            e["parity"] = ("tests/test_gpu_fp8.py::test_w8a16_chain_1280_vs_fp32_oracle: detections / chosen instance / "
                           f"cells / A* paths vs the fp32 oracle chain in the '{C5_REGIME}' regime this line runs")
        if ex == "c5_w8a8":
            e["form"] = "w8a8: e4m3 weights and activations on the block-scaled e4m3 MFMA"
            e["workload"] = ("C5 (BASELINE.json configs[4]) per GPU: YOLOv8m-seg 1280x1280, convs on e4m3 MFMA "
                             "(per-channel weight scales; activations stored as e4m3 with one calibrated power-of-two "
                             "scale per buffer), batch 8 = 64 across 8 GPUs, post-processing + grid / A* on GPU")
            e["parity"] = ("tests/test_gpu_fp8.py: op vs the same quantized operands; forward rel. L2 vs fp32; "
                           f"chain (detections / chosen instance / cells / A* paths) vs the fp32 oracle chain in the "
                           f"'{C5_REGIME}' regime this line runs")
        if prof:
            rl = m["roofline"]
            e["roofline"] = {k: rl[k] for k in ("achieved", "peak", "frac", "avg_launch_us", "traffic")}
        if ex == "bf16":
            e["parity"] = ("bf16 network: tests/test_gpu_chain.py compares its detections / chosen masks / cells / "
                           "A* paths with the fp32 oracle chain")
            if ing:
                e["ingest"] = ing
        extras[ex] = e

    if rank == 0:
        tag = {("s", 640): "C3", ("m", 1280): {"fp8": "C5 (fp8 MFMA)", "w8a16": "C5 (w8a16)"}.get(args.dtype, "C5 shape"),
               ("n", 640): "C2 shape (batched)"}.get((args.scale, args.res), "custom")
        H = W = args.res
        line = {
            "metric": "frames/sec end-to-end (seg+penalty+A*) at 640×640, 1/2/4/8 MI355X",  # BASELINE.json metric
            "value": round(main_res["value"], 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(main_res["ms_per_step"], 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (seeded uint8 frames; random-init yolov8%s-seg weights; planted nav masks when "
                    "the network yields none)" % args.scale,
            "config": {"workload": f"{tag}: YOLOv8{args.scale}-seg {H}x{W} {args.dtype} MFMA + post-processing + "
                                   "grid/penalty/protrusion/A* on GPU, end-to-end"
                                   + (" (natural regime: the synthetic weights yield no detections, so NMS / masks "
                                      "keep nothing and A* runs on planted masks; see extras.dense)"
                                      if args.regime == "natural" else ""),
                       "global_batch": world * B, "batch_per_gpu": B, "seq_len": None, "regime": args.regime,
                       "parallelism": f"frames sharded across {world} GPU(s), one process per GPU, no collective",
                       "overlap": (f"{args.seg_streams} network stream(s), {args.pipelines} batches in flight: "
                                   "consecutive forwards run concurrently; "
                                   "grid stage of batch k on its own stream under the following networks")
                       if run.overlap else "none",
                       "gflop_per_frame": round(main_res["gflop_alg"], 2),
                       "gflop_per_frame_executed": round(main_res["gflop_exec"] / B, 2)},
            "roofline": main_res.get("roofline"),
            "cpu_baseline": cpu,
            "ingest": ingest,
            "extras": extras,
            "astar_rounds_per_step": round(main_res["rounds"], 3),
            "unique_paths_last_batch": main_res["paths"],
            # host CPU seconds per wall second over the timed region (this process, all threads): a host that
            # spins (an OpenMP pool left busy-waiting) runs into the box's CPU quota and is throttled
            "host_cpu_per_wall": round(main_res["host_cpu"], 2),
        }
        print(json.dumps(line), flush=True)
    if dist:
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
