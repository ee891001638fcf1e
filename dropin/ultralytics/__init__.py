"""Drop-in import surface: with <repo>/dropin on PYTHONPATH, the reference's `from ultralytics import YOLO`
(main.py:6) resolves to vision_assist_amd.yolo.YOLO (the YOLOv8-seg forward on the MI355X kernels).  Put this
directory ahead of any installed ultralytics only for the process that runs the reference's main.py."""
from vision_assist_amd.yolo import YOLO, Masks, Results  # noqa: F401
