import sys
from pathlib import Path

_g = str(Path(__file__).resolve().parent / "golden")
if _g not in sys.path:
    sys.path.insert(0, _g)
