"""roctx ranges (cnmf_amd._trace): off by default, a no-op context either way on a
host without a profiler; the marker library loads from the image."""
import cnmf_amd
from cnmf_amd._trace import trace_range


def test_ranges_nest_and_toggle():
    was = cnmf_amd.tracing()
    try:
        cnmf_amd.tracing(True)
        with trace_range("outer"):
            with trace_range("inner"):
                pass
        assert cnmf_amd.tracing() in (True, False)  # True when a roctx library loaded
        cnmf_amd.tracing(False)
        assert cnmf_amd.tracing() is False
        with trace_range("off"):
            pass
    finally:
        cnmf_amd.tracing(was)
