#!/usr/bin/env python3
"""Drop-in for the reference `dist_model_tf_dense.py PATH` (same positional args)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from idc_models_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(["dist", "dense"] + sys.argv[1:]))
