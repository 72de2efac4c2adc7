"""Fluid BLAS on the gfx950 kernels: ``mul`` / ``matmul`` / ``fc`` for fp32 (and
fp16 / bf16 computed in fp32) run on the exact-fp32 MFMA GEMM of
``csrc/kernels/convnd.hip`` (``pa_sgemm``: fully strided operands, so transposed
views cost nothing; batched on blockIdx.z; split-K for under-filled shapes).
The bf16 model path uses the bf16 / fp8 GEMM of ``gemm.hip`` through
:mod:`paddle_amd.ops.fused` instead.

Backward: dA = alpha dC B^T and dB = alpha A^T dC on the same kernel; a weight
shared across a batch gets its gradient as ONE GEMM whose reduction runs over
the batch in registers (the kernel's k-batch).

Reference: operators/math/blas_impl.cu.h:27-200 (cublasSgemm / StridedBatched),
mul_op.cc, matmul_op.cc, fc_op.cc.
"""
from __future__ import annotations

import os

import torch

from . import convnd as _C
from ..autograd import tape as _tape  # noqa: E402

_ENABLED = os.environ.get("PADDLE_AMD_FLUID_BLAS", "1") != "0"


def supported(a, b):
    return (_ENABLED and _C.enabled() and a.is_cuda and b.is_cuda and a.dtype == b.dtype
            and a.dtype in (torch.float32, torch.float16, torch.bfloat16) and a.dim() in (2, 3) and b.dim() in (2, 3)
            and (b.dim() == 2 or (a.dim() == 3 and a.shape[0] == b.shape[0])) and a.shape[-1] == b.shape[-2]
            and a.numel() > 0 and b.numel() > 0 and (a.dim() == 2 or a.shape[0] <= 65535))


def _bmm(a, b, alpha=1.0):
    """a [Bt?, M, K], b [Bt?, K, N] (fp32, any strides) -> contiguous fp32 C [Bt?, M, N]."""
    M, K = a.shape[-2], a.shape[-1]
    N = b.shape[-1]
    if a.dim() == 2 and b.dim() == 2:
        c = torch.empty(M, N, dtype=torch.float32, device=a.device)
        _C.sgemm(a, a.stride(0), a.stride(1), b, b.stride(0), b.stride(1), c, N, M, N, K, alpha=alpha)
        return c
    if a.dim() == 3:
        Bt = a.shape[0]
        c = torch.empty(Bt, M, N, dtype=torch.float32, device=a.device)
        bsb = b.stride(0) if b.dim() == 3 else 0
        sbk, sbn = b.stride(-2), b.stride(-1)
        _C.sgemm(a, a.stride(1), a.stride(2), b, sbk, sbn, c, N, M, N, K, Z1=Bt,
                 bs1=(a.stride(0), bsb, M * N), alpha=alpha)
        return c
    raise ValueError("unsupported operand ranks")


def _shared_weight_grad(a, dc, alpha):
    """dB [K, N] = alpha * sum_bt a[bt]^T dc[bt] for a [Bt, M, K], dc [Bt, M, N]: one
    GEMM, reduction over (bt, m) with the batch on the kernel's k-batch."""
    Bt, M, K = a.shape
    N = dc.shape[-1]
    out = torch.empty(K, N, dtype=torch.float32, device=a.device)
    # A'(k, m) = a[bt][m][k]  -> rows k: sam = a.stride(2), sak = a.stride(1)
    # B'(m, n) = dc[bt][m][n] -> sbk = dc.stride(1), sbn = dc.stride(2)
    _C.sgemm(a, a.stride(2), a.stride(1), dc, dc.stride(1), dc.stride(2), out, N, K, N, M, kb=Bt,
             kbA=a.stride(0), kbB=dc.stride(0), alpha=alpha)
    return out


class _MatmulFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, alpha):
        dt = a.dtype
        af = a if dt == torch.float32 else a.float()
        bf = b if dt == torch.float32 else b.float()
        c = _bmm(af, bf, alpha)
        ctx.save_for_backward(af, bf)
        ctx.conf = (alpha, dt)
        return c if dt == torch.float32 else c.to(dt)

    @staticmethod
    def backward(ctx, dc):
        af, bf = ctx.saved_tensors
        alpha, dt = ctx.conf
        d = dc.float()
        da = db = None
        if ctx.needs_input_grad[0]:  # dA = alpha dC B^T (B^T as a strided view)
            da = _bmm(d, bf.transpose(-1, -2), alpha)
        if ctx.needs_input_grad[1]:
            if bf.dim() == 2 and af.dim() == 3:
                db = _shared_weight_grad(af, d, alpha)
            else:  # dB = alpha A^T dC
                db = _bmm(af.transpose(-1, -2), d, alpha)
        if dt != torch.float32:
            da = da.to(dt) if da is not None else None
            db = db.to(dt) if db is not None else None
        return da, db, None


def matmul(a, b, alpha=1.0):
    """C = alpha * a @ b for 2-D / 3-D operands (3-D b needs the same batch)."""
    return _tape.apply(_MatmulFn, a, b, float(alpha))


class _FcFn(torch.autograd.Function):
    """out = x @ w + bias[n]: the bias pre-broadcast into C, the GEMM accumulates on top
    (beta = 1); dbias = column sums of dC (pa_chan_sum)."""

    @staticmethod
    def forward(ctx, x, w, bias):
        dt = x.dtype
        xf = x if dt == torch.float32 else x.float()
        wf = w if dt == torch.float32 else w.float()
        M, K = xf.shape
        N = wf.shape[1]
        c = bias.float().reshape(1, N).expand(M, N).contiguous()
        _C.sgemm(xf, xf.stride(0), xf.stride(1), wf, wf.stride(0), wf.stride(1), c, N, M, N, K, beta=1.0)
        ctx.save_for_backward(xf, wf)
        ctx.conf = (dt, bias.dtype)
        return c if dt == torch.float32 else c.to(dt)

    @staticmethod
    def backward(ctx, dc):
        xf, wf = ctx.saved_tensors
        dt, bdt = ctx.conf
        d = dc.float().contiguous()
        da = _bmm(d, wf.t()) if ctx.needs_input_grad[0] else None
        dw = _bmm(xf.t(), d) if ctx.needs_input_grad[1] else None
        db = None
        if ctx.needs_input_grad[2]:
            M, N = d.shape
            db = torch.empty(N, dtype=torch.float32, device=d.device)
            _C.N.call("pa_chan_sum", _C.N.ptr(d), _C.N.ptr(db), M, N, 1, 0, _C.N.stream())
            db = db.to(bdt)
        return (da.to(dt) if da is not None else None, dw.to(dt) if dw is not None else None, db)


def fc(x2, w, bias):
    """x2 [M, K] @ w [K, N] + bias [N]."""
    return _tape.apply(_FcFn, x2, w, bias)
