"""vision_assist.PathAnalyser -> vision_assist_amd.PathAnalyser (drop-in import surface, dropin/vision_assist/__init__.py)."""
import sys

from vision_assist_amd import PathAnalyser as _impl

sys.modules[__name__] = _impl
