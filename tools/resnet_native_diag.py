"""Per-layer error of the native NHWC bf16 ResNet-50 path vs fp32 (and vs the ATen
bf16 path), plus a run-to-run determinism check of the native forward.

Prints one line per conv / BN module: rel-L2 error of its output against the fp32
model fed the same input.  Used to localise a loss mismatch in
tests/test_conv_gpu.py::test_resnet_native_matches_torch_path."""
import copy
import sys

import torch

import paddle_amd as paddle
from paddle_amd.ops import conv
from paddle_amd.ops import gemm as G

dev = "cuda"
paddle.seed(0)
torch.manual_seed(0)
base = paddle.vision.models.resnet50(num_classes=10, data_format="NHWC").to(dev)
g = torch.Generator(device=dev).manual_seed(1)
x = torch.randn(8, 64, 64, 3, generator=g, device=dev)


def capture(dtype, native):
    G.set_enabled(native)
    conv.set_enabled(native)
    outs = {}
    hooks = []
    m = copy.deepcopy(base).to(dtype)
    for name, mod in m.named_modules():
        if type(mod).__name__ in ("Conv2D", "BatchNorm2D", "MaxPool2D", "Linear", "BottleneckBlock"):
            hooks.append(mod.register_forward_hook(
                lambda mod, inp, out, name=name: outs.__setitem__(name, out.detach().float().clone())))
    with torch.no_grad():
        y = m(x.to(dtype)).float()
    for h in hooks:
        h.remove()
    G.set_enabled(True)
    conv.set_enabled(True)
    return y, outs


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


y32, o32 = capture(torch.float32, False)
ya, oa = capture(torch.bfloat16, False)
yn, on = capture(torch.bfloat16, True)
yn2, _ = capture(torch.bfloat16, True)
print(f"logits rel err: native {rel(yn, y32):.4e}  aten-bf16 {rel(ya, y32):.4e}  native run-to-run {rel(yn, yn2):.3e}")
worst = 0.0
for k in o32:
    en, ea = rel(on[k], o32[k]), rel(oa[k], o32[k])
    flag = "  <<<" if en > 3 * ea + 1e-2 else ""
    print(f"{k:40s} {tuple(o32[k].shape)!s:22s} native {en:.3e}  aten {ea:.3e}{flag}")
sys.stdout.flush()
