"""main.py runs unchanged (north_star: "drops into main.py unchanged"): with dropin/ on the path, the reference's
own import lines (main.py:6,8) resolve to this implementation -- checked on the text of those lines as main.py
has them (the file itself needs cv2 and a video, out of scope)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAIN_IMPORTS = ["from ultralytics import YOLO", "from vision_assist.FrameProcessor import FrameProcessor"]


def test_main_py_import_lines_resolve_to_vision_assist_amd():
    code = "\n".join(MAIN_IMPORTS + [
        "import vision_assist_amd.yolo as y, vision_assist_amd.FrameProcessor as f",
        "assert YOLO is y.YOLO and FrameProcessor is f.FrameProcessor",
        "from vision_assist.PathFinder import path_finder",
        "from vision_assist.models import Grid, Path, Coordinate",
        "from vision_assist.config import grid_size",
        "import vision_assist_amd.PathFinder as pf; assert path_finder is pf.path_finder",
        "print('ok')"])
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(REPO, "dropin"), REPO]))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().endswith("ok")
