"""utils/strict.py accounting on CPU tensors (WATCH_DEVICES extended for the test):
counted ATen kernels carry the framework call site that issued them under
FLAGS_strict_trace=1, and FLAGS_strict_native=1 turns them into errors."""
import pytest
import torch

from paddle_amd.utils import strict


@pytest.fixture
def watch_cpu(monkeypatch):
    monkeypatch.setattr(strict, "WATCH_DEVICES", {"cuda", "cpu"})
    monkeypatch.setenv("FLAGS_count_aten", "1")
    monkeypatch.setenv("FLAGS_strict_trace", "1")
    strict.reset()
    yield
    strict.reset()


def test_counted_kernel_names_its_framework_site(watch_cpu):
    from paddle_amd.ops import fused

    x = torch.ones(4)
    with strict.region("probe"):
        y = fused._scale_native(x, 3.0)
    assert torch.equal(y, torch.full((4,), 3.0))
    rep = strict.report()
    assert rep["aten_kernels"] == {"probe:mul": 1}, rep
    (site,) = rep["aten_sites"]["probe:mul"]
    assert site.startswith("paddle_amd/ops/fused.py:"), site


def test_strict_native_raises_inside_regions_only(watch_cpu, monkeypatch):
    monkeypatch.setenv("FLAGS_strict_native", "1")
    x = torch.ones(4)
    _ = x * 2  # outside every region: not watched
    with pytest.raises(strict.StrictNativeError):
        with strict.region("probe"):
            _ = x * 2
