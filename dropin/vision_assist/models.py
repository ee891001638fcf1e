"""vision_assist.models -> vision_assist_amd.models (drop-in import surface, dropin/vision_assist/__init__.py)."""
import sys

from vision_assist_amd import models as _impl

sys.modules[__name__] = _impl
