"""Composite networks (python/paddle/fluid/nets.py): simple_img_conv_pool, img_conv_group,
sequence_conv_pool, glu, scaled_dot_product_attention."""
from __future__ import annotations

from . import layers

__all__ = ["simple_img_conv_pool", "sequence_conv_pool", "glu", "scaled_dot_product_attention", "img_conv_group"]


def simple_img_conv_pool(input, num_filters, filter_size, pool_size, pool_stride, pool_padding=0,
                         pool_type="max", global_pooling=False, conv_stride=1, conv_padding=0, conv_dilation=1,
                         conv_groups=1, param_attr=None, bias_attr=None, act=None, use_cudnn=True, use_mkldnn=False):
    conv_out = layers.conv2d(input=input, num_filters=num_filters, filter_size=filter_size, stride=conv_stride,
                             padding=conv_padding, dilation=conv_dilation, groups=conv_groups,
                             param_attr=param_attr, bias_attr=bias_attr, act=act, use_cudnn=use_cudnn)
    return layers.pool2d(input=conv_out, pool_size=pool_size, pool_type=pool_type, pool_stride=pool_stride,
                         pool_padding=pool_padding, global_pooling=global_pooling, use_cudnn=use_cudnn)


def img_conv_group(input, conv_num_filter, pool_size, conv_padding=1, conv_filter_size=3, conv_act=None,
                   param_attr=None, conv_with_batchnorm=False, conv_batchnorm_drop_rate=0.0, pool_stride=1,
                   pool_type="max", use_cudnn=True, use_mkldnn=False):
    tmp = input
    n = len(conv_num_filter)

    def _l(obj):
        return obj if isinstance(obj, (list, tuple)) else [obj] * n

    conv_padding, conv_filter_size = _l(conv_padding), _l(conv_filter_size)
    param_attr, conv_with_batchnorm = _l(param_attr), _l(conv_with_batchnorm)
    conv_batchnorm_drop_rate = _l(conv_batchnorm_drop_rate)
    for i in range(n):
        local_act = conv_act
        if conv_with_batchnorm[i]:
            local_act = None
        tmp = layers.conv2d(input=tmp, num_filters=conv_num_filter[i], filter_size=conv_filter_size[i],
                            padding=conv_padding[i], param_attr=param_attr[i], act=local_act, use_cudnn=use_cudnn)
        if conv_with_batchnorm[i]:
            tmp = layers.batch_norm(input=tmp, act=conv_act)
            if abs(conv_batchnorm_drop_rate[i]) > 1e-5:
                tmp = layers.dropout(x=tmp, dropout_prob=conv_batchnorm_drop_rate[i])
    return layers.pool2d(input=tmp, pool_size=pool_size, pool_type=pool_type, pool_stride=pool_stride,
                         use_cudnn=use_cudnn)


def sequence_conv_pool(input, num_filters, filter_size, param_attr=None, act="sigmoid", pool_type="max"):
    conv_out = layers.sequence_conv(input=input, num_filters=num_filters, filter_size=filter_size,
                                    param_attr=param_attr, act=act)
    return layers.sequence_pool(input=conv_out, pool_type=pool_type)


def glu(input, dim=-1):
    a, b = layers.split(input, num_or_sections=2, dim=dim)
    return layers.elementwise_mul(x=a, y=layers.sigmoid(x=b))


def scaled_dot_product_attention(queries, keys, values, num_heads=1, dropout_rate=0.0):
    """Multi-head attention as matmul -> softmax -> matmul (nets.py:332-460)."""
    if num_heads > 1:
        def split_heads(x):
            hidden = x.shape[-1]
            r = layers.reshape(x, [0, 0, num_heads, hidden // num_heads])
            return layers.transpose(r, [0, 2, 1, 3])

        q, k, v = split_heads(queries), split_heads(keys), split_heads(values)
    else:
        q, k, v = queries, keys, values
    key_dim = keys.shape[-1] // num_heads
    scaled_q = layers.scale(x=q, scale=key_dim ** -0.5)
    product = layers.matmul(x=scaled_q, y=k, transpose_y=True)
    weights = layers.softmax(product)
    if dropout_rate:
        weights = layers.dropout(weights, dropout_prob=dropout_rate, is_test=False)
    ctx = layers.matmul(weights, v)
    if num_heads > 1:
        t = layers.transpose(ctx, [0, 2, 1, 3])
        ctx = layers.reshape(t, [0, 0, t.shape[2] * t.shape[3]])
    return ctx
