"""Hand-written gfx950 MFMA GEMM (csrc/kernels/gemm.hip) -- the matmul behind every
linear layer, replacing the vendor BLAS call of the reference
(paddle/fluid/operators/math/blas_impl.cu.h:27-200; mul_op.cc, matmul_op.cc, fc_op).

``gemm`` computes C (=|+=) alpha * A.B^T-style products where each operand is
either K-contiguous ("K-major", the reduction axis is the fastest one) or
MN-contiguous ("MN-major").  The three linear-layer products map onto it with no
transposed copies (Paddle weights are [in, out]):

* ``linear_fwd``  y  = x W        A = x  (K-major)   B = W  (MN-major)
* ``linear_dx``   dx = dy W^T     A = dy (K-major)   B = W  (K-major)
* ``linear_dw``   dW (+)= x^T dy  A = x  (MN-major)  B = dy (MN-major), fp32 out

Shapes: M, N, K multiples of 8, 16-B aligned row strides, each operand < 4 GiB;
``supported()`` says whether a call qualifies (callers fall back to torch only for
shapes the kernel does not cover, never silently on CUDA for covered ones).
"""
from __future__ import annotations

import os

import torch

from . import _native as _nat

_ENABLED = os.environ.get("PADDLE_AMD_GEMM", "1") != "0"
_LIMIT = 0xFFFFFF00


def enabled() -> bool:
    return _ENABLED


def set_enabled(flag: bool):
    global _ENABLED
    _ENABLED = bool(flag)


def supported(M, N, K, *mats) -> bool:
    if not _ENABLED or M % 8 or N % 8 or K % 8 or M <= 0 or N <= 0 or K <= 0:
        return False
    for t in mats:
        if not (t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 2 and t.stride(1) == 1
                and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0 and t.shape[0] * t.stride(0) * 2 < _LIMIT):
            return False
    return True


_SPLITK = os.environ.get("FLAGS_gemm_splitk", "1") not in ("0", "false", "False")
_NCU = []


def _num_cu():
    if not _NCU:
        _NCU.append(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count)
    return _NCU[0]


def split_k_for(M, N, K):
    """k-slices for a GEMM whose 256x256 tile count leaves the last round of the
    persistent grid mostly idle (320 tiles on 256 CUs run two rounds for 1.25 rounds of
    work).  Cost of s slices, in units of the ideal GEMM time: 1 / (filled fraction of
    the tile rounds) + the fp32 slab traffic of the slices and the summing pass,
    (4s + 2) bytes per output against the GEMM's 2K flops at ~1.45 PF / ~4.5 TB/s.  A
    split is taken when it saves >= 10 %; 1 = no split."""
    if not _SPLITK:
        return 1
    ncu = _num_cu()
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    if tiles >= 4 * ncu:
        return 1

    def eff(t):
        return t / (((t + ncu - 1) // ncu) * ncu)

    base = 1.0 / eff(tiles)
    best, best_s = base, 1
    for s in (2, 3, 4, 6, 8):
        if K // s < 1024:
            break
        c = 1.0 / eff(tiles * s) + (4 * s + 2) * 161.0 / K
        if c < best:
            best, best_s = c, s
    return best_s if best < 0.9 * base else 1


def _gemm_splitk(a, b, M, N, K, s, a_kmaj, b_kmaj, out, bias):
    """bf16 C = A.B (+ bias) as ``s`` k-slices into fp32 slabs and one summing pass."""
    ks = ((K + s - 1) // s + 63) // 64 * 64
    s = (K + ks - 1) // ks
    lda, ldb = a.stride(-2), b.stride(-2)
    part = torch.empty(s, M, N, dtype=torch.float32, device=a.device)
    rc = _nat.lib().pa_gemm(int(a_kmaj), int(b_kmaj), 1, _nat.ptr(a), _nat.ptr(b), _nat.ptr(part), None, M, N, ks,
                            lda, ldb, N, ks if a_kmaj else ks * lda, ks if b_kmaj else ks * ldb, M * N, s, 1.0, 0, K,
                            0, None, 0, _nat.stream())
    if rc != 0:
        raise RuntimeError(f"pa_gemm (split-K {s}) failed (rc={rc}) M={M} N={N} K={K}")
    _nat.call("pa_gemm_splitk_sum", _nat.ptr(part), s, M, N, _nat.ptr(bias), int(bias is not None and
                                                                                bias.dtype == torch.float32),
              _nat.ptr(out), out.stride(-2), _nat.stream())
    return out


def gemm(a, b, M, N, K, *, a_kmaj, b_kmaj, out=None, out_dtype=torch.bfloat16, bias=None, alpha=1.0,
         accumulate=False, batch=1, sA=0, sB=0, sC=0, ldc=None, k_total=0, atomic=False, grp=None, grp_mode=0):
    """Raw launcher.  ``a``/``b``: bf16 CUDA tensors with unit inner stride, row
    stride = their ld.  ``out``: [M, ldc] (bf16 or fp32) written or accumulated.
    A plain bf16-out GEMM with too few tiles for the chip runs split-K
    (:func:`split_k_for`)."""
    if (batch == 1 and not accumulate and not k_total and not atomic and grp is None and alpha == 1.0
            and (out is None or out.dtype == torch.bfloat16) and out_dtype == torch.bfloat16 and ldc is None):
        s = split_k_for(M, N, K)
        if s > 1:
            if out is None:
                out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
            return _gemm_splitk(a, b, M, N, K, s, a_kmaj, b_kmaj, out, bias)
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype, device=a.device) if batch == 1 else \
            torch.empty(batch, M, N, dtype=out_dtype, device=a.device)
        sC = M * N if batch > 1 else 0
    f32 = out.dtype == torch.float32
    if bias is not None and bias.dtype != out.dtype:
        bias = bias.to(out.dtype)
    lda, ldb = a.stride(-2), b.stride(-2)
    if ldc is None:
        ldc = out.stride(-2)
    rc = _nat.lib().pa_gemm(int(a_kmaj), int(b_kmaj), int(f32), _nat.ptr(a), _nat.ptr(b), _nat.ptr(out),
                           _nat.ptr(bias),
                         M, N, K, lda, ldb, ldc, sA, sB, sC, batch, float(alpha), int(accumulate), int(k_total),
                         int(atomic), _nat.ptr(grp), int(grp_mode), _nat.stream())
    if rc != 0:
        raise RuntimeError(f"pa_gemm failed (rc={rc}) M={M} N={N} K={K} a_kmaj={a_kmaj} b_kmaj={b_kmaj}")
    return out


def gemm_padded(a, b, M, N, K, *, a_kmaj, b_kmaj, out, accumulate=False):
    """:func:`gemm` for ragged M / N / K on 8-aligned row buffers (``pa_gemm_padded``):
    rows of ``a`` / ``b`` / ``out`` hold the extents rounded up to 8, the padding of a
    K-major operand past K (and of an MN-major ``a`` past M) is zero, and ``out``'s
    columns N .. round8(N) are written with zeros."""
    rc = _nat.lib().pa_gemm_padded(int(a_kmaj), int(b_kmaj), int(out.dtype == torch.float32), _nat.ptr(a),
                                   _nat.ptr(b), _nat.ptr(out), M, N, K, a.stride(-2), b.stride(-2), out.stride(-2),
                                   int(accumulate), _nat.stream())
    if rc != 0:
        raise RuntimeError(f"pa_gemm_padded failed (rc={rc}) M={M} N={N} K={K} a_kmaj={a_kmaj} b_kmaj={b_kmaj}")
    return out


EPI_SWIGLU_FWD, EPI_SWIGLU_BWD, EPI_ROPE = 1, 2, 3


def epi_supported(M, N, K, *mats) -> bool:
    """Fused-epilogue launches (``gemm_epi``): both operands K-major, K % 64 == 0."""
    return supported(M, N, K, *mats) and K % 64 == 0


def gemm_epi(epi, a, b, M, N, K, *, out, aux=None, cos=None, sin=None, rope_cols=0, rope_S=0):
    """C = A B^T (A [M, K], B [N, K], both K-major bf16) with a fused epilogue:

    * ``EPI_SWIGLU_FWD``: ``out`` [M, N] = the gate|up projection, gate and up
      interleaved in 16-column blocks; ``aux`` [M, N/2] receives silu(gate) * up;
    * ``EPI_SWIGLU_BWD``: the product is da [M, N]; ``aux`` [M, 2N] = gate|up in the
      same layout; ``out`` [M, 2N] receives (dgate, dup) at gate|up's positions;
    * ``EPI_ROPE``: ``out`` [M, N] with its first ``rope_cols`` columns rotated
      (neox) in 128-column heads by ``cos`` / ``sin`` [>= rope_S, 64] fp32 at position
      row % rope_S."""
    rc = _nat.lib().pa_gemm_epi(int(epi), _nat.ptr(a), _nat.ptr(b), _nat.ptr(out), _nat.ptr(aux),
                                aux.stride(0) if aux is not None else 0, M, N, K, a.stride(0), b.stride(0),
                                out.stride(0), _nat.ptr(cos), _nat.ptr(sin), int(rope_cols), int(rope_S),
                                _nat.stream())
    if rc != 0:
        raise RuntimeError(f"pa_gemm_epi failed (rc={rc}) epi={epi} M={M} N={N} K={K}")
    return out


def linear_fwd(x2, w, bias=None):
    """x2 [M, K] @ w [K, N] (+ bias) -> [M, N] bf16."""
    M, K = x2.shape
    Nn = w.shape[1]
    return gemm(x2, w, M, Nn, K, a_kmaj=True, b_kmaj=False, bias=bias)


def linear_dx(dy2, w):
    """dy2 [M, N] @ w[K, N]^T -> [M, K] bf16."""
    M, Nn = dy2.shape
    K = w.shape[0]
    return gemm(dy2, w, M, K, Nn, a_kmaj=True, b_kmaj=True)


def linear_dw(x2, dy2, out=None, accumulate=False):
    """x2[M, K]^T @ dy2[M, N] -> [K, N]; fp32 ``out`` (main_grad) accumulates."""
    M, K = x2.shape
    Nn = dy2.shape[1]
    if out is None:
        out = torch.empty(K, Nn, dtype=torch.float32, device=x2.device)
        accumulate = False
    return gemm(x2, dy2, K, Nn, M, a_kmaj=False, b_kmaj=False, out=out, accumulate=accumulate)


def matmul_nt(a, b):
    """a [M, K] @ b [N, K]^T -> [M, N] bf16."""
    M, K = a.shape
    return gemm(a, b, M, b.shape[0], K, a_kmaj=True, b_kmaj=True)


def gemm_splitk(a, b, M, N, K, *, a_kmaj, b_kmaj, out, accumulate=False, target_blocks=512):
    """C (+)= A.B with the reduction split over enough batches to fill the chip
    (tall-K products with few output tiles: conv weight gradients).  fp32 ``out``;
    every split adds its tile into ``out`` with float atomics in the GEMM epilogue
    (summation order varies run to run in the last bits)."""
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    S = max(1, min(target_blocks // max(tiles, 1), K // 256))
    if S <= 1:
        return gemm(a, b, M, N, K, a_kmaj=a_kmaj, b_kmaj=b_kmaj, out=out, accumulate=accumulate)
    Ks = ((K + S - 1) // S + 63) // 64 * 64
    S = (K + Ks - 1) // Ks
    if not accumulate:
        out.zero_()
    # k offset of one split, in elements: K-major operands advance along a row, MN-major by rows
    sA = Ks if a_kmaj else Ks * a.stride(-2)
    sB = Ks if b_kmaj else Ks * b.stride(-2)
    gemm(a, b, M, N, Ks, a_kmaj=a_kmaj, b_kmaj=b_kmaj, out=out, batch=S, sA=sA, sB=sB, sC=0, ldc=out.stride(0),
         k_total=K, atomic=True)
    return out


def group_table(offsets, total_rows):
    """int32 device row offsets [G + 1] -> the buffer a grouped-rows GEMM reads: the
    offsets followed by the tile table (group and row tile of every 256-row tile,
    ``pa_group_tile_table``), built on the device."""
    G = offsets.numel() - 1
    buf = torch.empty(G + 1 + (int(total_rows) + 255) // 256 + G, dtype=torch.int32, device=offsets.device)
    buf[:G + 1].copy_(offsets)
    rc = _nat.lib().pa_group_tile_table(_nat.ptr(buf), G, int(total_rows), _nat.stream())
    if rc != 0:
        raise RuntimeError(f"pa_group_tile_table failed (rc={rc}) G={G}")
    return buf


def grouped_rows(a, b, offsets, *, b_kmaj, out, bias=None):
    """Ragged grouped GEMM, one group per expert: rows [offsets[g], offsets[g+1]) of
    ``a`` (K-major, [rows, K]) times expert matrix ``b[g]`` (``b``: [G, K, N] MN-major or
    [G, N, K] K-major) into the same rows of ``out`` [rows, N].  ``offsets``: the
    int32 buffer of :func:`group_table` (G+1 row offsets + tile table), read only on
    the device (no host sync)."""
    G = b.shape[0]
    if b_kmaj:
        Nn, K = b.shape[1], b.shape[2]
    else:
        K, Nn = b.shape[1], b.shape[2]
    if G and a.shape[0] > 0:
        gemm(a, b[0], a.shape[0], Nn, K, a_kmaj=True, b_kmaj=b_kmaj, out=out, bias=bias, batch=G, sA=0,
             sB=b.stride(0), sC=0, ldc=out.stride(0), grp=offsets, grp_mode=1)
    return out


def grouped_dw(a, b, offsets, out, accumulate=True):
    """Per-group weight gradient out[g] (+)= a[rows_g]^T b[rows_g]: ``a`` [rows, M] and
    ``b`` [rows, N] (both MN-major), ``out`` [G, M, N] (fp32 main_grad or bf16)."""
    G, M, Nn = out.shape
    if G:
        gemm(a, b, M, Nn, 64, a_kmaj=False, b_kmaj=False, out=out[0], accumulate=accumulate, batch=G, sA=0, sB=0,
             sC=out.stride(0), ldc=out.stride(1), grp=offsets, grp_mode=2)
    return out
