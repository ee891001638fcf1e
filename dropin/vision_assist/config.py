"""vision_assist.config -> vision_assist_amd.config (drop-in import surface, dropin/vision_assist/__init__.py)."""
import sys

from vision_assist_amd import config as _impl

sys.modules[__name__] = _impl
