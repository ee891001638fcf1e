"""vision_assist.PathFinder -> vision_assist_amd.PathFinder (drop-in import surface, dropin/vision_assist/__init__.py)."""
import sys

from vision_assist_amd import PathFinder as _impl

sys.modules[__name__] = _impl
