"""ProtrusionDetector surface (reference: ProtrusionDetector.py).

The live path of the reference (ProtrusionDetector.py:419-439, 535: raster the
non-empty cells, top-most pixel row, runs split at gaps > grid_size // 4, run
centres) runs on the GPU inside ``nav_grid_kernel`` for every frame.  This
singleton keeps the reference's call signature ``(frame, grids, grid_lookup) ->
list[Coordinate]``: for the grids of the frame FrameProcessor holds it returns
that frame's device peaks; for grids built elsewhere it runs the device grid
stage on the frame they imply (FrameProcessor.device_frame_for) and returns its
peaks.  The defect / quadrilateral code the reference comments out (:445-504)
is not built.
"""
from __future__ import annotations

from typing import ClassVar, Optional

from .models import Coordinate


class ProtrusionDetector:
    _instance: ClassVar[Optional["ProtrusionDetector"]] = None
    _initialized: bool = False

    def __new__(cls, debug: bool = False, imshow: bool = False):
        if cls._instance is None:
            cls._instance = super().__new__(cls)
            cls._instance.debug = debug
            cls._instance.imshow = imshow
        return cls._instance

    def __init__(self, debug: bool = False, imshow: bool = False):
        if not self._initialized:
            self._initialized = True
            self.frame = None
            self.grids = None
            self.height = 0
            self.width = 0
            self.binary = None
            self.frames_processed = 0

    def __call__(self, frame, grids, grid_lookup) -> list[Coordinate]:
        from .FrameProcessor import FrameProcessor
        fp = FrameProcessor._instance
        self.frame = frame
        self.grids = grids
        self.height, self.width = frame.shape[0], frame.shape[1]
        self.frames_processed += 1
        st = fp._state if fp is not None else None
        if st is None or grids is not st.grids:
            from .FrameProcessor import device_frame_for
            st = device_frame_for(grids, grid_lookup, self.height, self.width)
        return st.peaks()
