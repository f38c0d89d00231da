"""roctx tracing helpers (idc_models_amd/utils/trace.py): a no-op unless IDC_ROCTX=1, real roctx
ranges (balanced push/pop) when enabled and the ROCm roctx library is present."""
from idc_models_amd.utils import trace


def test_disabled_is_noop(monkeypatch):
    monkeypatch.delenv("IDC_ROCTX", raising=False)
    with trace.range("x"):
        trace.mark("m")
    assert not trace.enabled()


def test_enabled_ranges_nest(monkeypatch):
    monkeypatch.setenv("IDC_ROCTX", "1")
    with trace.range("outer"):
        with trace.range("inner"):
            trace.mark("m")
    # depth returned by roctxRangePushA is the nesting level (>= 0) when the library loaded
    lib = trace._load()
    if lib is not None:
        d = lib.roctxRangePushA(b"probe")
        lib.roctxRangePop()
        assert d >= 0
