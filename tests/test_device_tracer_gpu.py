"""In-process kernel tracing on rocprofiler-sdk (utils/device_tracer.py,
csrc/tracer/device_tracer.cc; the reference's CUPTI DeviceTracer,
platform/device_tracer.cc:98-121).  The tool has to be registered before the HIP
runtime starts, so the check runs in a fresh process with FLAGS_device_tracer=1."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import json, sys, torch
import paddle_amd
from paddle_amd.utils import device_tracer as dt, profiler as P
from paddle_amd.ops import gemm as G
assert dt.available(), dt.error()
a = torch.randn(512, 256, device="cuda").to(torch.bfloat16)
b = torch.randn(384, 256, device="cuda").to(torch.bfloat16)
torch.cuda.synchronize()
P.start("All")
with P.RecordEvent("my_gemm"):
    c = G.gemm(a, b, 512, 384, 256, a_kmaj=True, b_kmaj=True)
with P.RecordEvent("my_add"):
    d = c.float() + 1.0
prof = P.profile_dict()
recs = P.kernel_records()
P.stop(profile_path=None)
ref = a.float() @ b.float().t()
assert (c.float() - ref).abs().max().item() < 0.05 * ref.abs().max().item()
gpu = [e for e in prof["events"] if e["type"] == "GPUKernel"]
host = {e["name"]: e for e in prof["events"] if e["type"] == "CPU"}
print(json.dumps({"recs": [{k: r[k] for k in ("name", "op", "dur_ns", "device", "grid", "block", "lds")} for r in recs],
                  "gpu": gpu, "host": host, "dropped": dt.dropped()}))
"""


def test_device_tracer_records_kernels_with_op_ranges():
    env = dict(os.environ, FLAGS_device_tracer="1", PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-c", SCRIPT], cwd=REPO, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    recs = out["recs"]
    gemm = [x for x in recs if "gemm_kernel" in x["name"]]
    assert gemm, [x["name"] for x in recs]
    g = gemm[0]
    assert g["op"] == "my_gemm" and g["dur_ns"] > 0 and g["device"] == 0
    assert g["block"][0] == 512 and g["lds"] > 64 * 1024  # 8 waves, LDS-staged tiles
    # the add ran inside its own range; no kernel of the window is unattributed
    assert any(x["op"] == "my_add" for x in recs)
    assert out["dropped"] == 0
    # the GPU track of the profile is the kernel records, on the host clock: each
    # kernel starts after its range began on the host
    assert len(out["gpu"]) == len(recs)
    k = [e for e in out["gpu"] if "gemm_kernel" in e["name"]][0]
    assert k["start_ns"] >= out["host"]["my_gemm"]["start_ns"] - 1_000_000
