import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "mm-admm_amd", "python"))

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    return GOLDEN


def circle_mesh(name):
    """Mesh files the reference committed (Experiments/Results/BaseCircle*), copied to golden/."""
    import oracle_py

    d = 3 if name.startswith("3D") else 2
    sub = "BaseCircle3D" if d == 3 else "BaseCircle"
    b = os.path.join(GOLDEN, sub, name)
    return oracle_py.Mesh.read(d, b + "triangles.txt", b + "points.txt", b + "mask.txt")
