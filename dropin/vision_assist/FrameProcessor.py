"""vision_assist.FrameProcessor -> vision_assist_amd.FrameProcessor (drop-in import surface, dropin/vision_assist/__init__.py)."""
import sys

from vision_assist_amd import FrameProcessor as _impl

sys.modules[__name__] = _impl
