"""v2 composite networks (reference v2/networks.py over
trainer_config_helpers/networks.py)."""
from . import layer
from . import pooling as P


def simple_img_conv_pool(input, filter_size, num_filters, pool_size, num_channel=None, pool_stride=1, act=None,
                         pool_type=None, **kw):
    c = layer.img_conv(input, filter_size, num_filters, num_channels=num_channel, act=act)
    return layer.img_pool(c, pool_size, stride=pool_stride, pool_type=pool_type or P.Max())


def sequence_conv_pool(input, context_len, hidden_size, **kw):
    from .. import fluid
    from ._core import guard

    with guard():
        c = fluid.layers.sequence_conv(input, hidden_size, filter_size=context_len, act="tanh")
        return fluid.layers.sequence_pool(c, "MAX")


def simple_lstm(input, size, **kw):
    from .. import fluid
    from ._core import guard

    with guard():
        proj = fluid.layers.fc(input, size * 4)
        h, _ = fluid.layers.dynamic_lstm(proj, size * 4)
    return h
