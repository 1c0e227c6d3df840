"""pytest configuration: the `gpu` marker and shared fixtures.

`-m "not gpu"` runs everywhere (oracle vs golden vectors, host logic, C-ABI
exports, multi-rank gloo tests of the segmented orchestration);
`-m gpu` needs an MI355X and calls the HIP library through the C ABI.
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (runs the HIP kernels)")


def golden_cases(algo=None):
    with open(os.path.join(GOLDEN, "index.json")) as f:
        idx = json.load(f)
    return [c for c in idx if algo is None or c["algo"] == algo]


def load_golden(case):
    with np.load(os.path.join(GOLDEN, case["file"]), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def gpu_target():
    import hpx_amd
    n = hpx_amd.compute.get_device_count()
    if n == 0:
        pytest.fail("no GPU visible: -m gpu tests need an MI355X")
    return hpx_amd.target(0)
