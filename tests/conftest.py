import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libgta.so")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


_MANIFEST = []


def load_manifest():
    """tests/golden/manifest.json, read once: test modules parametrize over its entries at
    collection time (one test per golden stream / candidate list, no placeholder skips)."""
    if not _MANIFEST:
        import json
        with open(os.path.join(GOLDEN, "manifest.json")) as f:
            _MANIFEST.append(json.load(f))
    return _MANIFEST[0]


@pytest.fixture(scope="session")
def manifest():
    return load_manifest()


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


# Full-size GPU checks first: the metric kernel at Reddit size, the BASELINE-config
# layers and the multi-rank bench run before the many small kernel-form tests, so an early `-x`
# stop in a small test cannot hide them.  Order inside each group is kept.
_FIRST = ("test_gpu_metric.py", "test_gpu_configs.py", "test_gpu_distributed.py")


def pytest_collection_modifyitems(config, items):
    def rank(item):
        name = os.path.basename(str(item.fspath))
        return _FIRST.index(name) if name in _FIRST else len(_FIRST)
    items[:] = sorted(items, key=rank)  # stable: the rest keep their collection order
