"""Shared test setup.

* Registers the `gpu` marker: tests that need an MI355X (`pytest -m gpu`); everything else runs on
  the CPU (`pytest -m "not gpu"`).
* Puts the package directory (union-thesis-slam_amd/, the analogue of the reference's repo root on
  sys.path) and oracle/ on sys.path.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "union-thesis-slam_amd")
GOLD = os.path.join(REPO, "tests", "golden")
for p in (PKG, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct GPU (MI355X) and the HIP library")
    config.addinivalue_line("markers", "slow: CPU test taking more than ~20 s")


def load_lounge(i, color=True):
    """Lounge frame i from the committed fixture copy, ingested like grid_demo1.py:80-84."""
    from PIL import Image
    d = np.array(Image.open(os.path.join(GOLD, "lounge", "frame-%06d.depth.png" % i)))
    depth = d.astype(float) / 1000.0
    depth[depth == 65.535] = 0
    pose = np.loadtxt(os.path.join(GOLD, "lounge", "frame-%06d.pose.txt" % i))
    rgb = None
    if color:
        rgb = np.array(Image.open(os.path.join(GOLD, "lounge", "frame-%06d.color.jpg" % i)).convert("RGB"))
    return d, depth, rgb, pose


def lounge_intrinsics():
    return np.loadtxt(os.path.join(GOLD, "lounge", "camera-intrinsics.txt"), delimiter=" ")


@pytest.fixture(scope="session")
def gold():
    return GOLD
