import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libotmatch's HIP kernels)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def small_graph(tmp_path_factory):
    """5 x 5 km synthetic city (config 1 extract)."""
    from reporter_amd import synth
    d = tmp_path_factory.mktemp("graphs")
    return synth.make_graph(str(d / "small.otmg"), width_m=5000, height_m=5000)


@pytest.fixture(scope="session")
def rural_graph(tmp_path_factory):
    """Sparse highway-heavy 40 x 40 km extract in the config-4 style."""
    from reporter_amd import synth
    d = tmp_path_factory.mktemp("graphs")
    g = dict(synth.CONFIGS[4]["graph"])
    g.update(width_m=40000, height_m=40000)
    return synth.make_graph(str(d / "rural.otmg"), **g)


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.lib()
    return pyoracle


def equal_results(a, b, what=""):
    """Field-wise equality of two result sets (oracle dict vs product Results)."""
    import numpy.testing as npt
    ta = a["traces"] if isinstance(a, dict) else a.traces
    tb = b["traces"] if isinstance(b, dict) else b.traces
    for f in ta.dtype.names:
        npt.assert_array_equal(ta[f], tb[f], err_msg="%s traces.%s" % (what, f))
    sa = a["segments"] if isinstance(a, dict) else a.segments
    sb = b["segments"] if isinstance(b, dict) else b.segments
    assert len(sa) == len(sb), "%s segment count %d != %d" % (what, len(sa), len(sb))
    for f in sa.dtype.names:
        npt.assert_array_equal(sa[f], sb[f], err_msg="%s segments.%s" % (what, f))
    ra = a["reports"] if isinstance(a, dict) else a.reports
    rb = b["reports"] if isinstance(b, dict) else b.reports
    assert len(ra) == len(rb), "%s report count" % what
    for f in ra.dtype.names:
        npt.assert_array_equal(ra[f], rb[f], err_msg="%s reports.%s" % (what, f))
    wa = a["way_ids"] if isinstance(a, dict) else a.way_ids
    wb = b["way_ids"] if isinstance(b, dict) else b.way_ids
    npt.assert_array_equal(wa, wb, err_msg="%s way_ids" % what)


@pytest.fixture
def results_equal():
    return equal_results
