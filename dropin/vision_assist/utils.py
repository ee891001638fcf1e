"""vision_assist.utils -> vision_assist_amd.utils (drop-in import surface, dropin/vision_assist/__init__.py)."""
import sys

from vision_assist_amd import utils as _impl

sys.modules[__name__] = _impl
