"""Drop-in import surface for the reference's own package name: with <repo>/dropin on PYTHONPATH,
`from vision_assist.FrameProcessor import FrameProcessor` (main.py:8) and the other hot-path modules resolve to
vision_assist_amd.  Modules outside the hot path (MockCamera: video I/O, out of scope) are found in the reference
checkout named by VISION_ASSIST_REF, which is appended to this package's search path."""
import os

_ref = os.environ.get("VISION_ASSIST_REF")
if _ref and os.path.isdir(_ref):
    __path__.append(_ref)  # noqa: F821 -- the package's own search path
