"""Import of the host-only native modules (``_idc_data``, ``_idc_paillier``, ``_idc_h5``).

``IDC_HOST_EXT_DIR=<dir>`` loads them from ``<dir>`` instead of the package (the
AddressSanitizer / UBSan / ThreadSanitizer builds of ``tools/sanitize_host.py``), under the same
module name, so the code and tests that use them run unchanged against the instrumented build.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys
import sysconfig


def import_host_ext(name: str):
    full = f"idc_models_amd.{name}"
    d = os.environ.get("IDC_HOST_EXT_DIR")
    if d:
        path = os.path.join(d, name + sysconfig.get_config_var("EXT_SUFFIX"))
        if os.path.exists(path):
            if full in sys.modules:
                return sys.modules[full]
            spec = importlib.util.spec_from_file_location(full, path)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            sys.modules[full] = mod
            return mod
    return importlib.import_module(full)
