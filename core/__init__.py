"""Drop-in `core` package: the reference's engine surface (core/engine.py, core/inference.py,
core/config.py, core/models/model_loader.py) backed by the MI355X HIP runtime in
video-caption-algorithm_amd/vcap."""
import sys as _sys
from pathlib import Path as _Path

_PKG = _Path(__file__).resolve().parents[1] / "video-caption-algorithm_amd"
if str(_PKG) not in _sys.path:
    _sys.path.insert(0, str(_PKG))
