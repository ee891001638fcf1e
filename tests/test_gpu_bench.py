"""bench.py keeps the driver's contract: one JSON line with the BASELINE.json metric, a positive value, the
roofline and cpu_baseline objects.  Small run (batch 8, 2 steps) in a child process."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_contract_line():
    out = subprocess.run([sys.executable, "bench.py", "--batch", "8", "--steps", "2", "--warmup", "1",
                          "--cpu-sample", "2"], cwd=REPO, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        assert d["metric"] == json.load(f)["metric"]
    assert d["value"] > 0 and d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["unit"] == "frames/s" and d["higher_is_better"] is True and d["scaling"] == "weak"
    r = d["roofline"]
    assert r["bound"] == "mfma" and r["unit"] == "TFLOP/s" and 0 < r["frac"] < 1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    c = d["cpu_baseline"]
    assert c["value"] > 0 and c["kind"] == "port" and c["cores"] >= 1
    assert d["config"]["workload"].startswith("C3")
    # the reference's precision (args.yaml half: false): f32 products as exact bf16 term products on the bf16 MFMA,
    # priced against the bf16 peak; the f32-MFMA view beside it
    assert d["dtype"] == "f32" and r["peak"] == 2500.0 and r["f32_equivalent"]["peak"] == 157.3
    assert abs(r["f32_equivalent"]["achieved"] * 6 - r["achieved"]) < 0.02 * r["achieved"]
    assert set(d["extras"]) == {"bf16", "dense", "dense_box", "c5", "c5_w8a8", "c4", "c2", "dropin", "dealer"}
    # C4's own shape (one frame per GPU per step), C2 latency, the drop-in FrameProcessor.__call__ rate
    assert d["extras"]["c4"]["batch_per_gpu"] == 1 and d["extras"]["c4"]["value"] > 0
    assert d["extras"]["c2"]["seg_only"]["median_ms"] > 0 and d["extras"]["c2"]["end_to_end"]["median_ms"] > 0
    assert d["extras"]["dropin"]["value"] > 0 and d["extras"]["dropin"]["calls_with_answer"] > 0
    assert d["extras"]["bf16"]["roofline"]["peak"] == 2500.0 and d["extras"]["dense"]["dtype"] == "f32"
    assert d["extras"]["c5"]["dtype"] == "w8a16" and d["extras"]["c5"]["roofline"]["peak"] == 2500.0
    assert d["extras"]["c5_w8a8"]["dtype"] == "fp8" and d["extras"]["c5_w8a8"]["roofline"]["peak"] == 5000.0
    assert "grid_stage_ms_per_frame" in c and "path+analyser" in c["stage_ms_per_frame"]


def test_bench_gpus_2_starts_its_own_ranks():
    """The driver's command form `python bench.py --gpus N` (no torch.distributed.run): bench.py starts N ranks
    itself (here both share cuda:0, LOCAL_RANK % device_count) and relays rank 0's line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--batch", "8", "--steps", "2", "--warmup", "1",
                          "--extras", "none", "--no-ingest"], cwd=REPO, capture_output=True, text=True,
                         timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 16 and d["config"]["batch_per_gpu"] == 8
    assert d["value"] > 0 and d["scaling"] == "weak" and d["cpu_baseline"] is None
