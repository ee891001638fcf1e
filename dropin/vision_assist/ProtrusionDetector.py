"""vision_assist.ProtrusionDetector -> vision_assist_amd.ProtrusionDetector (drop-in import surface, dropin/vision_assist/__init__.py)."""
import sys

from vision_assist_amd import ProtrusionDetector as _impl

sys.modules[__name__] = _impl
