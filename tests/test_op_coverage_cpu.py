"""Every operator type the reference registers (REGISTER_OPERATOR /
REGISTER_OP_WITHOUT_GRADIENT / REGISTER_ACTIVATION_OP under paddle/fluid/operators)
has a kernel here, except the TensorRT engine op (no gfx950 backend; README
non-goals)."""
import glob
import os
import re

import pytest

import paddle_amd.operators  # noqa: F401
from paddle_amd.framework import registry as R

REF = "/root/reference/paddle/fluid/operators"
_PAT = re.compile(r"REGISTER_(?:OPERATOR|OP_WITHOUT_GRADIENT|ACTIVATION_OP)\(\s*([a-z][a-zA-Z0-9_]*)")


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_every_reference_op_type_is_registered():
    names = set()
    for f in glob.glob(os.path.join(REF, "**", "*.cc"), recursive=True):
        with open(f, errors="ignore") as fh:
            names.update(_PAT.findall(fh.read()))
    fwd = {n for n in names if not n.endswith("_grad")} - {"tensorrt_engine"}
    missing = sorted(n for n in fwd if n not in R.OP_REGISTRY)
    assert len(fwd) > 150
    assert not missing, missing
