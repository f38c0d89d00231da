#!/usr/bin/env python3
"""Drop-in for the reference `secure_fed_model.py PATH ROUNDS PERCENT`."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from idc_models_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(["secure"] + sys.argv[1:]))
