import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _reset_amp_state():
    yield
    try:
        from apex_example_amd.amp import amp as _amp
        from apex_example_amd.amp._amp_state import _amp_state

        if getattr(_amp_state, "handle", None) is not None:
            _amp.deinit()
            _amp_state.handle = None
    except Exception:
        pass
