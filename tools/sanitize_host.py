#!/usr/bin/env python3
"""Host-code sanitizer runs (SURVEY §5 race detection / sanitizers).

Builds the host-only native modules — the threaded PNG loader with its pinned prefetch ring
(``csrc/data/loader.cpp``), the GMP Paillier vector ops (``csrc/fed/paillier_gmp.cpp``) and the
libhdf5 Keras weight I/O (``csrc/ckpt/h5io.cpp``) — with AddressSanitizer + UndefinedBehavior
Sanitizer, and the loader with ThreadSanitizer, then runs their CPU tests in a process that
preloads the matching system sanitizer runtime and loads the instrumented modules through
``IDC_HOST_EXT_DIR``.  Any report aborts the run (halt_on_error), so exit 0 means clean.  GPU code
is not sanitized (no GPU ASan / xnack on this pool).

    python tools/sanitize_host.py [address|thread ...]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tools.build_native import build_sanitized, sanitize_dir  # noqa: E402

RUNS = {
    "address": {"runtime": "libasan.so",
                "tests": ["tests/test_native_data.py", "tests/test_paillier_native.py", "tests/test_ckpt.py"],
                "mods": ["_idc_data", "_idc_paillier", "_idc_h5"],
                "env": {"ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1:abort_on_error=0",
                        "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}},
    "thread": {"runtime": "libtsan.so",
               "tests": ["tests/test_native_data.py"],
               "mods": ["_idc_data"],
               "env": {"TSAN_OPTIONS": "halt_on_error=1:report_signal_unsafe=0"}},
}

CHECK = r"""
import os, sys, torch
from idc_models_amd.utils.hostext import import_host_ext
for name in sys.argv[1:]:
    m = import_host_ext(name)
    assert os.path.realpath(m.__file__).startswith(os.path.realpath(os.environ["IDC_HOST_EXT_DIR"])), m.__file__
print("instrumented:", " ".join(sys.argv[1:]))
"""


def run(kind: str) -> int:
    cfg = RUNS[kind]
    d = build_sanitized(kind, verbose=False)
    rt = subprocess.run(["gcc", f"-print-file-name={cfg['runtime']}"], capture_output=True, text=True).stdout.strip()
    env = dict(os.environ, IDC_HOST_EXT_DIR=d, LD_PRELOAD=rt, **cfg["env"])
    r = subprocess.run([sys.executable, "-c", CHECK] + cfg["mods"], cwd=ROOT, env=env, capture_output=True, text=True)
    if r.returncode != 0:
        print(f"[{kind}] instrumented modules did not load:\n{r.stderr[-3000:]}")
        return r.returncode or 1
    print(f"[{kind}] {r.stdout.strip()}")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider"] + cfg["tests"],
                       cwd=ROOT, env=env, capture_output=True, text=True)
    tail = (r.stdout + r.stderr)[-3000:]
    print(f"[{kind}] rc={r.returncode}\n{tail}")
    return r.returncode


def main(argv):
    kinds = argv or list(RUNS)
    rc = 0
    for k in kinds:
        rc = rc or run(k)
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
