"""``paddle.vision.models``: LeNet, ResNet (18/34/50/101/152), VGG, MobileNetV2.

ResNet-50 is BASELINE.json's conv/BN configuration ("ResNet-50 bf16 on one
MI355X"; the reference's Fluid number is 105.84 img/s on a TITAN X,
doc/fluid/new_docs/advanced_usage/benchmark.rst:117 -- model definition
benchmark/fluid/models/resnet.py).  MI355X layout: ``data_format="NHWC"`` keeps
activations channels-last so MIOpen runs its NHWC bf16 MFMA convolutions with no
layout transposes; BatchNorm folds into the same layout.  Parameter names follow
paddle.vision (``conv1``, ``bn1``, ``layer1.0.conv1`` ..., ``fc``) with Paddle's
``[in, out]`` Linear weights.
"""
from __future__ import annotations

import torch

from .. import nn
from ..ops import conv as _conv


class LeNet(nn.Layer):
    def __init__(self, num_classes=10):
        super().__init__()
        self.num_classes = num_classes
        self.features = nn.Sequential(
            nn.Conv2D(1, 6, 3, stride=1, padding=1), nn.ReLU(), nn.MaxPool2D(2, 2),
            nn.Conv2D(6, 16, 5, stride=1, padding=0), nn.ReLU(), nn.MaxPool2D(2, 2))
        if num_classes > 0:
            self.fc = nn.Sequential(nn.Linear(400, 120), nn.Linear(120, 84), nn.Linear(84, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.num_classes > 0:
            x = self.fc(torch.flatten(x, 1))
        return x


def _fusable(bn, x):
    return isinstance(bn, nn.layer_bn_types()) and bn.training and not bn._use_global_stats \
        and bn._data_format == "NHWC" and _conv.supported_bn(x)


def _bn_relu(bn, x, residual=None):
    """relu(bn(x) [+ residual]); one fused HIP pass (BatchNorm with the residual add
    and the ReLU in its epilogue, the ReLU mask applied in its backward) for NHWC
    bf16 training on the GPU."""
    if _fusable(bn, x) and (residual is None or residual.shape == x.shape):
        return _conv.batch_norm_nhwc_train(x, bn.weight, bn.bias, bn._mean, bn._variance, bn._momentum,
                                           bn._epsilon, relu=True, residual=residual)
    y = bn(x)
    return torch.relu(y if residual is None else y + residual)


def _conv_direct(conv, x):
    """The conv layer may be run by conv2d_nhwc directly (NHWC native path, no hooks)."""
    pad = conv._padding
    return (isinstance(conv, nn.Conv2D) and conv._data_format == "NHWC" and conv._padding_mode == "zeros"
            and not conv._forward_pre_hooks and not conv._forward_hooks
            and (isinstance(pad, int) or (isinstance(pad, (list, tuple)) and len(pad) == 2))
            and _conv.supported_conv(x, conv.weight, conv._stride, pad, conv._dilation, conv._groups))


def _conv_bn_relu(conv, bn, x, residual=None, relu=True):
    """relu(bn(conv(x)) [+ residual]) (``relu=False``: bn(conv(x))).  On the native
    NHWC path the BatchNorm batch statistics come from the conv's epilogue, so the
    BN forward makes one pass over the conv output instead of two."""
    if _conv_direct(conv, x) and _fusable(bn, x):
        rm = bn._mean
        st = {"shift": rm if (rm is not None and rm.dtype == torch.float32 and rm.is_contiguous()) else None}
        y = _conv.conv2d_nhwc(x, conv.weight, conv.bias, conv._stride, conv._padding, conv._dilation, stats=st)
        if residual is None or residual.shape == y.shape:
            return _conv.batch_norm_nhwc_train(y, bn.weight, bn.bias, bn._mean, bn._variance, bn._momentum,
                                               bn._epsilon, relu=relu, residual=residual, stats=st)
        return _bn_relu(bn, y, residual) if relu else bn(y)
    if not relu:
        return bn(conv(x))
    return _bn_relu(bn, conv(x), residual)


def _downsample(ds, x):
    """The projection shortcut: Sequential(conv, bn) through the conv-statistics path."""
    mods = list(ds.children()) if isinstance(ds, nn.Sequential) else None
    if (mods is not None and len(mods) == 2 and isinstance(mods[1], nn.layer_bn_types())
            and not ds._forward_pre_hooks and not ds._forward_hooks):
        return _conv_bn_relu(mods[0], mods[1], x, relu=False)
    return ds(x)


class BasicBlock(nn.Layer):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None, data_format="NCHW"):
        super().__init__()
        bn = norm_layer or nn.BatchNorm2D
        self.conv1 = nn.Conv2D(inplanes, planes, 3, padding=1, stride=stride, bias_attr=False,
                               data_format=data_format)
        self.bn1 = bn(planes, data_format=data_format)
        self.relu = nn.ReLU()
        self.conv2 = nn.Conv2D(planes, planes, 3, padding=1, bias_attr=False, data_format=data_format)
        self.bn2 = bn(planes, data_format=data_format)
        self.downsample = downsample

    def forward(self, x):
        identity = x
        out = _conv_bn_relu(self.conv1, self.bn1, x)
        if self.downsample is not None:
            identity = _downsample(self.downsample, x)
        return _conv_bn_relu(self.conv2, self.bn2, out, identity)


class BottleneckBlock(nn.Layer):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None, data_format="NCHW"):
        super().__init__()
        bn = norm_layer or nn.BatchNorm2D
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = nn.Conv2D(inplanes, width, 1, bias_attr=False, data_format=data_format)
        self.bn1 = bn(width, data_format=data_format)
        self.conv2 = nn.Conv2D(width, width, 3, padding=dilation, stride=stride, groups=groups, dilation=dilation,
                               bias_attr=False, data_format=data_format)
        self.bn2 = bn(width, data_format=data_format)
        self.conv3 = nn.Conv2D(width, planes * self.expansion, 1, bias_attr=False, data_format=data_format)
        self.bn3 = bn(planes * self.expansion, data_format=data_format)
        self.relu = nn.ReLU()
        self.downsample = downsample

    def forward(self, x):
        identity = x
        out = _conv_bn_relu(self.conv1, self.bn1, x)
        out = _conv_bn_relu(self.conv2, self.bn2, out)
        if self.downsample is not None:
            identity = _downsample(self.downsample, x)
        return _conv_bn_relu(self.conv3, self.bn3, out, identity)


class ResNet(nn.Layer):
    def __init__(self, block, depth=50, width=64, num_classes=1000, with_pool=True, groups=1, data_format="NCHW"):
        super().__init__()
        layer_cfg = {18: [2, 2, 2, 2], 34: [3, 4, 6, 3], 50: [3, 4, 6, 3], 101: [3, 4, 23, 3], 152: [3, 8, 36, 3]}
        layers = layer_cfg[depth]
        self.groups, self.base_width = groups, width
        self.num_classes, self.with_pool = num_classes, with_pool
        self.data_format = data_format
        self.inplanes = 64
        self.dilation = 1
        self.conv1 = nn.Conv2D(3, self.inplanes, 7, stride=2, padding=3, bias_attr=False, data_format=data_format)
        self.bn1 = nn.BatchNorm2D(self.inplanes, data_format=data_format)
        self.relu = nn.ReLU()
        self.maxpool = nn.MaxPool2D(3, 2, 1, data_format=data_format)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D((1, 1), data_format=data_format)
        if num_classes > 0:
            self.fc = nn.Linear(512 * block.expansion, num_classes)

    def _make_layer(self, block, planes, blocks, stride=1):
        df = self.data_format
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(nn.Conv2D(self.inplanes, planes * block.expansion, 1, stride=stride, bias_attr=False,
                                           data_format=df),
                                 nn.BatchNorm2D(planes * block.expansion, data_format=df))
        layers = [block(self.inplanes, planes, stride, down, self.groups, self.base_width, data_format=df)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups, base_width=self.base_width,
                                data_format=df))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(_bn_relu(self.bn1, self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if self.with_pool:
            x = self.avgpool(x)
        if self.num_classes > 0:
            x = self.fc(torch.flatten(x, 1))
        return x


def _resnet(block, depth, pretrained=False, **kw):
    if pretrained:
        raise ValueError("no network access: pretrained weights are unavailable")
    return ResNet(block, depth, **kw)


def resnet18(pretrained=False, **kw):
    return _resnet(BasicBlock, 18, pretrained, **kw)


def resnet34(pretrained=False, **kw):
    return _resnet(BasicBlock, 34, pretrained, **kw)


def resnet50(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 50, pretrained, **kw)


def resnet101(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 101, pretrained, **kw)


def resnet152(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 152, pretrained, **kw)


def wide_resnet50_2(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 50, pretrained, width=128, **kw)


def resnext50_32x4d(pretrained=False, **kw):
    return _resnet(BottleneckBlock, 50, pretrained, width=4, groups=32, **kw)


class VGG(nn.Layer):
    def __init__(self, features, num_classes=1000, with_pool=True, data_format="NCHW"):
        super().__init__()
        self.features = features
        self.num_classes, self.with_pool = num_classes, with_pool
        self.data_format = data_format
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D((7, 7), data_format=data_format)
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Linear(512 * 7 * 7, 4096), nn.ReLU(), nn.Dropout(),
                                            nn.Linear(4096, 4096), nn.ReLU(), nn.Dropout(),
                                            nn.Linear(4096, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.avgpool(x)
        if self.num_classes > 0:
            if self.data_format == "NHWC":   # classifier weights keep the NCHW flatten order
                x = x.permute(0, 3, 1, 2)
            x = self.classifier(torch.flatten(x, 1))
        return x


def _vgg_features(cfg, batch_norm=False, data_format="NCHW"):
    layers, c = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2D(2, 2, data_format=data_format))
        else:
            layers.append(nn.Conv2D(c, v, 3, padding=1, data_format=data_format))
            if batch_norm:
                layers.append(nn.BatchNorm2D(v, data_format=data_format))
            layers.append(nn.ReLU())
            c = v
    return nn.Sequential(*layers)


_VGG = {16: [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
        19: [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"],
        11: [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
        13: [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"]}


def vgg16(pretrained=False, batch_norm=False, **kw):
    return VGG(_vgg_features(_VGG[16], batch_norm, kw.get("data_format", "NCHW")), **kw)


def vgg19(pretrained=False, batch_norm=False, **kw):
    return VGG(_vgg_features(_VGG[19], batch_norm, kw.get("data_format", "NCHW")), **kw)


def vgg11(pretrained=False, batch_norm=False, **kw):
    return VGG(_vgg_features(_VGG[11], batch_norm, kw.get("data_format", "NCHW")), **kw)


def vgg13(pretrained=False, batch_norm=False, **kw):
    return VGG(_vgg_features(_VGG[13], batch_norm, kw.get("data_format", "NCHW")), **kw)


class _InvertedResidual(nn.Layer):
    def __init__(self, inp, oup, stride, expand_ratio):
        super().__init__()
        hidden = int(round(inp * expand_ratio))
        self.use_res = stride == 1 and inp == oup
        layers = []
        if expand_ratio != 1:
            layers += [nn.Conv2D(inp, hidden, 1, bias_attr=False), nn.BatchNorm2D(hidden), nn.ReLU6()]
        layers += [nn.Conv2D(hidden, hidden, 3, stride, 1, groups=hidden, bias_attr=False), nn.BatchNorm2D(hidden),
                   nn.ReLU6(), nn.Conv2D(hidden, oup, 1, bias_attr=False), nn.BatchNorm2D(oup)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.conv(x) if self.use_res else self.conv(x)


class MobileNetV2(nn.Layer):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        cfg = [[1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2], [6, 96, 3, 1], [6, 160, 3, 2],
               [6, 320, 1, 1]]
        inp = int(32 * scale)
        self.last = int(1280 * max(1.0, scale))
        feats = [nn.Conv2D(3, inp, 3, 2, 1, bias_attr=False), nn.BatchNorm2D(inp), nn.ReLU6()]
        for t, c, n, s in cfg:
            out = int(c * scale)
            for i in range(n):
                feats.append(_InvertedResidual(inp, out, s if i == 0 else 1, t))
                inp = out
        feats += [nn.Conv2D(inp, self.last, 1, bias_attr=False), nn.BatchNorm2D(self.last), nn.ReLU6()]
        self.features = nn.Sequential(*feats)
        self.with_pool, self.num_classes = with_pool, num_classes
        if with_pool:
            self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Dropout(0.2), nn.Linear(self.last, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.pool2d_avg(x)
        if self.num_classes > 0:
            x = self.classifier(torch.flatten(x, 1))
        return x


def mobilenet_v2(pretrained=False, scale=1.0, **kw):
    return MobileNetV2(scale, **kw)
