"""pytest configuration: `gpu` marker, import paths, build-once fixtures."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gnss-sdr.ru_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def _make(*args):
    subprocess.run(["make", "-s", *args], check=True, cwd=ROOT)


@pytest.fixture(scope="session")
def gc():
    """The product package (libgnsscorr.so built in-tree)."""
    so = os.path.join(PKG, "gnsscorr", "libgnsscorr.so")
    if not os.path.exists(so):
        _make("-C", PKG)
    import gnsscorr
    return gnsscorr


@pytest.fixture(scope="session")
def oracle():
    import osg_oracle
    if not os.path.exists(osg_oracle.ORACLE_SO):
        _make("-C", os.path.join(ROOT, "oracle"))
    return osg_oracle


@pytest.fixture(scope="session")
def gpu(gc):
    if gc.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return gc
