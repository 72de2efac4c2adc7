import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def pytest_sessionfinish(session, exitstatus):
    """FLAGS_count_aten / FLAGS_strict_native runs: write the native-dispatch census
    (ATen kernels left per region and op, native ops executed) to PA_ATEN_REPORT."""
    path = os.environ.get("PA_ATEN_REPORT")
    if not path:
        return
    try:
        import json

        from paddle_amd.utils import strict

        rep = strict.report()
        rep["aten_kernels"] = dict(sorted(rep["aten_kernels"].items(), key=lambda kv: -kv[1]))
        with open(path, "w") as f:
            json.dump(rep, f, indent=1)
    except Exception as e:  # pragma: no cover - diagnostics only
        print("aten report failed:", e)
