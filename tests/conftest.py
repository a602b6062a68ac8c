import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950); run with -m gpu")


def has_reference():
    return os.path.isdir(os.path.join(REFERENCE, "sampling_based_planner"))


@pytest.fixture(scope="session")
def planner_model():
    from manipulator_mujoco_amd import models
    return models.load("planner_scene", 0.05)


@pytest.fixture(scope="session")
def all_models():
    from manipulator_mujoco_amd import models
    return {k: models.load(k, 0.05) for k in models.BUNDLES}
