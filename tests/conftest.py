import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "vector-store-text_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvsg.so on cuda:0)")
    config.addinivalue_line("markers", "slow: larger parity case")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def load_golden(name):
    import numpy as np
    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    return {k: z[k] for k in z.files}


def golden_inputs(g):
    """Regenerate a fixture's inputs from its seeds (inputs are never committed)."""
    from vsg import datagen as G
    gen = str(g["gen"])
    n, d, nq = int(g["n"]), int(g["dim"]), int(g["nq"])
    if gen == "uint8":
        return G.uint8_valued(n, d, int(g["base_seed"])), G.uint8_valued(nq, d, int(g["query_seed"]))
    ms = int(g["model_seed"])
    return (G.clustered(n, d, int(g["base_seed"]), ms), G.clustered(nq, d, int(g["query_seed"]), ms))
