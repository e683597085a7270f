import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "time-warp_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


# every replica-mode GPU test runs under each kernel geometry (TW_GEOMETRY)
GEOMETRIES = ["dense", "sparse", "half", "wave", "narrow", "compact"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtimewarp.so on cuda:0)")
    config.addinivalue_line("markers", "slow: larger CPU cases")
    config.addinivalue_line("markers", "one_geometry: a GPU test whose kernel choice is not a replica geometry "
                                       "(LP mode) or that pins its own: run once")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def engine_mod():
    from timewarp import engine

    engine.load_library()
    return engine


@pytest.fixture(autouse=True)
def tw_geometry(request, monkeypatch):
    """GPU tests run under every kernel geometry (dense: 256 replicas per
    workgroup; sparse: 16 per workgroup with the 768-entry on-chip queue;
    half: the dense layout as 8 waves of 32 lanes)."""
    g = getattr(request, "param", None)
    if g is not None:
        monkeypatch.setenv("TW_GEOMETRY", g)
    return g


def pytest_generate_tests(metafunc):
    if "tw_geometry" in metafunc.fixturenames and metafunc.definition.get_closest_marker("gpu"):
        if metafunc.definition.get_closest_marker("one_geometry"):
            metafunc.parametrize("tw_geometry", [None], indirect=True)
        else:
            metafunc.parametrize("tw_geometry", GEOMETRIES, indirect=True)
