"""Shared fixtures.  `gpu` marks tests that need an MI355X (run via gpurun)."""
import importlib.util
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs under gpurun")


def load_pkg():
    """Import rgbd-slam_amd (a directory name that is not a Python identifier)."""
    name = "rgbd_slam_amd"
    if name in sys.modules:
        return sys.modules[name]
    pkg_dir = os.path.join(ROOT, "rgbd-slam_amd")
    spec = importlib.util.spec_from_file_location(name, os.path.join(pkg_dir, "__init__.py"),
                                                  submodule_search_locations=[pkg_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def pkg():
    return load_pkg()


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    oracle_lib.lib()
    return oracle_lib


_SEQ_CACHE = {}


def synth_seq(n, seed=3, preset="fr1", start=0):
    import synth
    key = (n, seed, preset, start)
    if key not in _SEQ_CACHE:
        _SEQ_CACHE[key] = synth.sequence(n, seed=seed, preset=preset, start=start)
    return _SEQ_CACHE[key]


@pytest.fixture(scope="session")
def seq_fr1():
    return synth_seq(4, seed=3, preset="fr1")


@pytest.fixture(scope="session")
def seq_fr3():
    return synth_seq(3, seed=11, preset="fr3")
