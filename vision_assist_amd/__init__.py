"""vision_assist_amd -- MI355X-native implementation of vision-assist's per-frame hot path.

Python host surface (same class/module names as the reference: FrameProcessor,
PathFinder, PenaltyCalculator, ProtrusionDetector, models, utils, config) over
hand-written HIP kernels for gfx950 in ``libva355.so`` (C ABI: include/va355.h).
"""
__version__ = "0.1.0"
