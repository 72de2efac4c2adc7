"""paddle.nn.utils helpers."""
from __future__ import annotations

import torch

from ..optimizer.clip import ClipGradByGlobalNorm


def clip_grad_norm_(parameters, max_norm, norm_type=2.0, error_if_nonfinite=False):
    ps = [p for p in (parameters if not torch.is_tensor(parameters) else [parameters]) if p.grad is not None]
    if norm_type != 2.0:
        return torch.nn.utils.clip_grad_norm_(ps, max_norm, norm_type, error_if_nonfinite)
    c = ClipGradByGlobalNorm(max_norm)
    n = c.global_norm([(p, p.grad) for p in ps])
    c._clip([(p, p.grad) for p in ps])
    return n


def clip_grad_value_(parameters, clip_value):
    torch.nn.utils.clip_grad_value_(parameters, clip_value)


def parameters_to_vector(parameters, name=None):
    return torch.nn.utils.parameters_to_vector(parameters)


def vector_to_parameters(vec, parameters, name=None):
    torch.nn.utils.vector_to_parameters(vec, parameters)


def weight_norm(layer, name="weight", dim=0):
    return torch.nn.utils.parametrizations.weight_norm(layer, name, dim)


def spectral_norm(layer, name="weight", n_power_iterations=1, eps=1e-12, dim=None):
    return torch.nn.utils.parametrizations.spectral_norm(layer, name, n_power_iterations, eps, dim)
