"""vision_assist.PenaltyCalculator -> vision_assist_amd.PenaltyCalculator (drop-in import surface, dropin/vision_assist/__init__.py)."""
import sys

from vision_assist_amd import PenaltyCalculator as _impl

sys.modules[__name__] = _impl
