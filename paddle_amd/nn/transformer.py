"""paddle.nn Transformer family and recurrent layers.

``MultiHeadAttention`` keeps Paddle's ``q_proj/k_proj/v_proj/out_proj`` Linear
sub-layers (``[in, out]`` weights) and runs the attention core on the gfx950
flash-attention kernel when there is no explicit mask / dropout (bf16, head_dim
64/128 on the GPU); otherwise the masked path uses SDPA.  ``LSTM``/``GRU``/
``SimpleRNN`` keep Paddle's parameter names (``weight_ih_l{k}``, ``weight_hh_l{k}``,
``bias_ih_l{k}``, ``bias_hh_l{k}``; ``direction="bidirect"`` adds the ``_reverse``
set) and gate order.  On the GPU, LSTM runs every layer/direction on the
persistent gfx950 kernel (``ops/rnn.py``: one launch per sequence, W_hh resident in
registers; 1.9x MIOpen at B 32, H 512, T 833) when H is 128/256/512/1024 and the
batch is <= 128; other shapes and GRU/SimpleRNN use MIOpen through PyTorch-ROCm.
"""
from __future__ import annotations

import copy

import torch

from .. import ops
from . import functional as F
from .layer import Dropout, Layer, LayerList, LayerNorm, Linear


class MultiHeadAttention(Layer):
    def __init__(self, embed_dim, num_heads, dropout=0.0, kdim=None, vdim=None, need_weights=False,
                 weight_attr=None, bias_attr=None):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.head_dim = embed_dim // num_heads
        self.dropout, self.need_weights = dropout, need_weights
        self.q_proj = Linear(embed_dim, embed_dim, weight_attr, bias_attr)
        self.k_proj = Linear(kdim or embed_dim, embed_dim, weight_attr, bias_attr)
        self.v_proj = Linear(vdim or embed_dim, embed_dim, weight_attr, bias_attr)
        self.out_proj = Linear(embed_dim, embed_dim, weight_attr, bias_attr)

    def forward(self, query, key=None, value=None, attn_mask=None, cache=None, is_causal=False):
        key = query if key is None else key
        value = key if value is None else value
        B, Sq, _ = query.shape
        Sk = key.shape[1]
        q = self.q_proj(query).reshape(B, Sq, self.num_heads, self.head_dim)
        k = self.k_proj(key).reshape(B, Sk, self.num_heads, self.head_dim)
        v = self.v_proj(value).reshape(B, Sk, self.num_heads, self.head_dim)
        drop = self.dropout if self.training else 0.0
        if self.need_weights:
            s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) / self.head_dim ** 0.5
            if attn_mask is not None:
                s = s + attn_mask if attn_mask.dtype != torch.bool else s.masked_fill(~attn_mask, float("-inf"))
            w = torch.softmax(s, -1)
            w = F.dropout(w, drop, training=self.training)
            o = torch.einsum("bhqk,bkhd->bqhd", w, v.float()).to(query.dtype)
            return self.out_proj(o.reshape(B, Sq, self.embed_dim)), w
        fast = attn_mask is None and drop == 0.0 and (not query.is_cuda or (query.dtype == torch.bfloat16 and
                                                                             self.head_dim in (64, 128)))
        if fast:
            o = ops.flash_attention(q, k, v, causal=is_causal)
        else:
            o = F.scaled_dot_product_attention(q, k, v, attn_mask, drop, is_causal, self.training)
        return self.out_proj(o.reshape(B, Sq, self.embed_dim))


class TransformerEncoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout=0.1, activation="relu", attn_dropout=None,
                 act_dropout=None, normalize_before=False, weight_attr=None, bias_attr=None, layer_norm_eps=1e-5):
        super().__init__()
        attn_dropout = dropout if attn_dropout is None else attn_dropout
        act_dropout = dropout if act_dropout is None else act_dropout
        self.normalize_before = normalize_before
        self.self_attn = MultiHeadAttention(d_model, nhead, attn_dropout, weight_attr=weight_attr, bias_attr=bias_attr)
        self.linear1 = Linear(d_model, dim_feedforward, weight_attr, bias_attr)
        self.dropout = Dropout(act_dropout)
        self.linear2 = Linear(dim_feedforward, d_model, weight_attr, bias_attr)
        self.norm1 = LayerNorm(d_model, layer_norm_eps)
        self.norm2 = LayerNorm(d_model, layer_norm_eps)
        self.dropout1 = Dropout(dropout)
        self.dropout2 = Dropout(dropout)
        self.activation = getattr(F, activation)

    def forward(self, src, src_mask=None, cache=None):
        res = src
        if self.normalize_before:
            src = self.norm1(src)
        src = res + self.dropout1(self.self_attn(src, src, src, src_mask))
        if not self.normalize_before:
            src = self.norm1(src)
        res = src
        if self.normalize_before:
            src = self.norm2(src)
        src = res + self.dropout2(self.linear2(self.dropout(self.activation(self.linear1(src)))))
        if not self.normalize_before:
            src = self.norm2(src)
        return src


class TransformerEncoder(Layer):
    def __init__(self, encoder_layer, num_layers, norm=None):
        super().__init__()
        self.layers = LayerList([encoder_layer if i == 0 else copy.deepcopy(encoder_layer)
                                 for i in range(num_layers)])
        self.norm = norm

    def forward(self, src, src_mask=None, cache=None):
        for l in self.layers:
            src = l(src, src_mask)
        return self.norm(src) if self.norm is not None else src


class TransformerDecoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout=0.1, activation="relu", attn_dropout=None,
                 act_dropout=None, normalize_before=False, weight_attr=None, bias_attr=None, layer_norm_eps=1e-5):
        super().__init__()
        attn_dropout = dropout if attn_dropout is None else attn_dropout
        act_dropout = dropout if act_dropout is None else act_dropout
        self.normalize_before = normalize_before
        self.self_attn = MultiHeadAttention(d_model, nhead, attn_dropout, weight_attr=weight_attr, bias_attr=bias_attr)
        self.cross_attn = MultiHeadAttention(d_model, nhead, attn_dropout, weight_attr=weight_attr,
                                             bias_attr=bias_attr)
        self.linear1 = Linear(d_model, dim_feedforward, weight_attr, bias_attr)
        self.dropout = Dropout(act_dropout)
        self.linear2 = Linear(dim_feedforward, d_model, weight_attr, bias_attr)
        self.norm1 = LayerNorm(d_model, layer_norm_eps)
        self.norm2 = LayerNorm(d_model, layer_norm_eps)
        self.norm3 = LayerNorm(d_model, layer_norm_eps)
        self.dropout1, self.dropout2, self.dropout3 = Dropout(dropout), Dropout(dropout), Dropout(dropout)
        self.activation = getattr(F, activation)

    def _blk(self, x, norm, fn):
        if self.normalize_before:
            return x + fn(norm(x))
        return norm(x + fn(x))

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, cache=None):
        causal = tgt_mask is None
        tgt = self._blk(tgt, self.norm1, lambda t: self.dropout1(self.self_attn(t, t, t, tgt_mask,
                                                                                is_causal=causal)))
        tgt = self._blk(tgt, self.norm2, lambda t: self.dropout2(self.cross_attn(t, memory, memory, memory_mask)))
        tgt = self._blk(tgt, self.norm3,
                        lambda t: self.dropout3(self.linear2(self.dropout(self.activation(self.linear1(t))))))
        return tgt


class TransformerDecoder(Layer):
    def __init__(self, decoder_layer, num_layers, norm=None):
        super().__init__()
        self.layers = LayerList([decoder_layer if i == 0 else copy.deepcopy(decoder_layer)
                                 for i in range(num_layers)])
        self.norm = norm

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, cache=None):
        for l in self.layers:
            tgt = l(tgt, memory, tgt_mask, memory_mask)
        return self.norm(tgt) if self.norm is not None else tgt


class Transformer(Layer):
    def __init__(self, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6, dim_feedforward=2048,
                 dropout=0.1, activation="relu", attn_dropout=None, act_dropout=None, normalize_before=False,
                 weight_attr=None, bias_attr=None, custom_encoder=None, custom_decoder=None):
        super().__init__()
        enc = TransformerEncoderLayer(d_model, nhead, dim_feedforward, dropout, activation, attn_dropout, act_dropout,
                                      normalize_before, weight_attr, bias_attr)
        dec = TransformerDecoderLayer(d_model, nhead, dim_feedforward, dropout, activation, attn_dropout, act_dropout,
                                      normalize_before, weight_attr, bias_attr)
        self.encoder = custom_encoder or TransformerEncoder(enc, num_encoder_layers,
                                                            LayerNorm(d_model) if normalize_before else None)
        self.decoder = custom_decoder or TransformerDecoder(dec, num_decoder_layers,
                                                            LayerNorm(d_model) if normalize_before else None)

    def forward(self, src, tgt, src_mask=None, tgt_mask=None, memory_mask=None):
        return self.decoder(tgt, self.encoder(src, src_mask), tgt_mask, memory_mask)

    @staticmethod
    def generate_square_subsequent_mask(length):
        return torch.triu(torch.full((length, length), float("-inf")), 1)


# ------------------------------------------------------------------------ RNNs
class _RNNBase(Layer):
    _mode = None

    def __init__(self, input_size, hidden_size, num_layers=1, direction="forward", time_major=False, dropout=0.0,
                 activation="tanh", weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None, bias_hh_attr=None,
                 name=None):
        super().__init__(name)
        bidir = direction in ("bidirect", "bidirectional")
        kw = dict(input_size=input_size, hidden_size=hidden_size, num_layers=num_layers, bias=True,
                  batch_first=not time_major, dropout=dropout, bidirectional=bidir)
        if self._mode == "RNN":
            kw["nonlinearity"] = activation
        self.rnn = getattr(torch.nn, self._mode)(**kw)
        self.time_major, self.num_directions = time_major, 2 if bidir else 1
        self.hidden_size, self.num_layers = hidden_size, num_layers

    def _persistent_ok(self, x):
        import os

        from ..ops import rnn as R

        if self._mode != "LSTM" or os.environ.get("PADDLE_AMD_PERSISTENT_LSTM", "1") == "0":
            return False
        B = x.shape[1 if self.time_major else 0]
        return R.persistent_ok(x, self.hidden_size, B)

    def _persistent_lstm(self, x, initial_states, lens):
        """Every layer/direction on the persistent gfx950 LSTM kernel (ops/rnn.py);
        same outputs as torch's (padded positions zeroed, h_n/c_n = last states)."""
        from ..ops import rnn as R

        inp = x if self.time_major else x.transpose(0, 1)
        T = inp.shape[0]
        h_n, c_n = [], []
        for layer in range(self.num_layers):
            outs = []
            for d in range(self.num_directions):
                sfx = f"_l{layer}" + ("_reverse" if d else "")
                w_ih = getattr(self.rnn, "weight_ih" + sfx).t()
                w_hh = getattr(self.rnn, "weight_hh" + sfx).t()
                b = getattr(self.rnn, "bias_ih" + sfx) + getattr(self.rnn, "bias_hh" + sfx)
                k = layer * self.num_directions + d
                h0 = initial_states[0][k] if initial_states is not None else None
                c0 = initial_states[1][k] if initial_states is not None else None
                xi = R.reverse_padded(inp, lens) if d else inp
                hs, h, c = R.lstm(xi, w_ih, w_hh, b, h0, c0, lens=lens)
                outs.append(R.reverse_padded(hs, lens) if d else hs)
                h_n.append(h)
                c_n.append(c)
            inp = torch.cat(outs, -1) if len(outs) > 1 else outs[0]
            if self.rnn.dropout and self.training and layer < self.num_layers - 1:
                inp = torch.nn.functional.dropout(inp, self.rnn.dropout)
        out = inp
        if lens is not None:
            m = torch.arange(T, device=out.device).unsqueeze(1) < lens.to(out.device).unsqueeze(0)
            out = out * m.unsqueeze(-1).to(out.dtype)
        if not self.time_major:
            out = out.transpose(0, 1)
        return out, (torch.stack(h_n), torch.stack(c_n))

    def forward(self, inputs, initial_states=None, sequence_length=None):
        if self._persistent_ok(inputs):
            return self._persistent_lstm(inputs, initial_states, sequence_length)
        x = inputs
        if sequence_length is not None:
            x = torch.nn.utils.rnn.pack_padded_sequence(x, sequence_length.cpu(), batch_first=not self.time_major,
                                                        enforce_sorted=False)
        out, st = self.rnn(x, initial_states)
        if sequence_length is not None:
            out, _ = torch.nn.utils.rnn.pad_packed_sequence(out, batch_first=not self.time_major,
                                                            total_length=inputs.shape[0 if self.time_major else 1])
        return out, st

    # Paddle parameter names == torch's (weight_ih_l0, ..., *_reverse): state dicts map 1:1
    def state_dict(self, *a, **k):
        sd = super().state_dict(*a, **k)
        return type(sd)((key.replace("rnn.", "", 1), v) for key, v in sd.items())

    def load_state_dict(self, sd, strict=True):
        return super().load_state_dict({("rnn." + k if not k.startswith("rnn.") else k): v for k, v in sd.items()},
                                       strict)

    set_state_dict = load_state_dict


class SimpleRNN(_RNNBase):
    _mode = "RNN"


class LSTM(_RNNBase):
    _mode = "LSTM"


class GRU(_RNNBase):
    _mode = "GRU"


class LSTMCell(Layer):
    def __init__(self, input_size, hidden_size, weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None,
                 bias_hh_attr=None, name=None):
        super().__init__(name)
        self.cell = torch.nn.LSTMCell(input_size, hidden_size)
        self.hidden_size = hidden_size

    def forward(self, inputs, states=None):
        h, c = self.cell(inputs, states)
        return h, (h, c)


class GRUCell(Layer):
    def __init__(self, input_size, hidden_size, weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None,
                 bias_hh_attr=None, name=None):
        super().__init__(name)
        self.cell = torch.nn.GRUCell(input_size, hidden_size)
        self.hidden_size = hidden_size

    def forward(self, inputs, states=None):
        h = self.cell(inputs, states)
        return h, h


class SimpleRNNCell(Layer):
    def __init__(self, input_size, hidden_size, activation="tanh", weight_ih_attr=None, weight_hh_attr=None,
                 bias_ih_attr=None, bias_hh_attr=None, name=None):
        super().__init__(name)
        self.cell = torch.nn.RNNCell(input_size, hidden_size, nonlinearity=activation)
        self.hidden_size = hidden_size

    def forward(self, inputs, states=None):
        h = self.cell(inputs, states)
        return h, h
