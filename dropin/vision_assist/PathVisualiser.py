"""vision_assist.PathVisualiser -> vision_assist_amd.PathVisualiser (drop-in import surface, dropin/vision_assist/__init__.py)."""
import sys

from vision_assist_amd import PathVisualiser as _impl

sys.modules[__name__] = _impl
