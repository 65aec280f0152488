"""Drop-in CLIs of the reference (run from this package's directory):

    python -m src.semi_supervised_training --strong-data-dir ... --weak-data-dir ...
    python -m src.supervised_training --strong-data-dir ...
    python -m src.feature_extraction --data-dir ...

As in the reference (src/semi_supervised_training.py:19-20), the training
CLIs import `training.*`, so this directory is put on sys.path; the parent
directory provides the `ssip` host runtime over libssip_hip.so.
"""
import sys as _sys
from pathlib import Path as _Path

for _p in (_Path(__file__).resolve().parent, _Path(__file__).resolve().parents[1]):
    if str(_p) not in _sys.path:
        _sys.path.insert(0, str(_p))
