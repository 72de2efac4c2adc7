"""The v1 config parser's protobuf output: TrainerConfig / ModelConfig / LayerConfig /
ParameterConfig / OptimizationConfig / DataConfig (reference proto/TrainerConfig.proto,
ModelConfig.proto, ParameterConfig.proto, DataConfig.proto), built while a config runs.

The reference ``config_parser.parse_config`` turns a v1 config into a TrainerConfig
message for the legacy GradientMachine.  Here the DSL builds a Fluid program
(``trainer_config_helpers``), and this module records, for every layer call of the
config, the LayerConfig the reference would emit -- the same default names
(``__fc_layer_0__``, ``___fc_layer_0__.w0`` / ``.wbias``), layer types, sizes,
activation names, inputs and parameters -- so ``TrainerConfig.proto()`` serialises
a wire-compatible TrainerConfig and ``dump_config`` prints its text form
(reference python/paddle/utils/dump_config.py).  ``parameter_name_map`` maps the
v1 parameter names to the Fluid parameters that hold them.

The wire codec is a schema-driven proto2 encoder / decoder (varint, 64-bit, 32-bit,
length-delimited; unknown fields skipped on decode) plus a text-format printer and
parser; tests/test_v1_config_proto_cpu.py checks the output against the reference's
own expected protostr files.
"""
from __future__ import annotations

import inspect
import re
import struct

# ---------------------------------------------------------------- schemas
# field: (name, number, kind, repeated); kind: scalar type name or a message name
_S = {
    "ParameterUpdaterHookConfig": [("type", 1, "string", 0), ("sparsity_ratio", 2, "double", 0)],
    "ParameterConfig": [
        ("name", 1, "string", 0), ("size", 2, "uint64", 0), ("learning_rate", 3, "double", 0),
        ("momentum", 4, "double", 0), ("initial_mean", 5, "double", 0), ("initial_std", 6, "double", 0),
        ("decay_rate", 7, "double", 0), ("decay_rate_l1", 8, "double", 0), ("dims", 9, "uint64", 1),
        ("device", 10, "int32", 0), ("initial_strategy", 11, "int32", 0), ("initial_smart", 12, "bool", 0),
        ("num_batches_regularization", 13, "int32", 0), ("is_sparse", 14, "bool", 0), ("format", 15, "string", 0),
        ("sparse_remote_update", 16, "bool", 0), ("gradient_clipping_threshold", 17, "double", 0),
        ("is_static", 18, "bool", 0), ("para_id", 19, "uint64", 0),
        ("update_hooks", 20, "ParameterUpdaterHookConfig", 1), ("need_compact", 21, "bool", 0),
        ("sparse_update", 22, "bool", 0), ("is_shared", 23, "bool", 0),
        ("parameter_block_size", 24, "uint64", 0)],
    "SliceConfig": [("start", 1, "uint32", 0), ("end", 2, "uint32", 0)],
    "ImageConfig": [("channels", 2, "uint32", 0), ("img_size", 8, "uint32", 0), ("img_size_y", 9, "uint32", 0),
                    ("img_size_z", 10, "uint32", 0)],
    "ConvConfig": [
        ("filter_size", 1, "uint32", 0), ("channels", 2, "uint32", 0), ("stride", 3, "uint32", 0),
        ("padding", 4, "uint32", 0), ("groups", 5, "uint32", 0), ("filter_channels", 6, "uint32", 0),
        ("output_x", 7, "uint32", 0), ("img_size", 8, "uint32", 0), ("caffe_mode", 9, "bool", 0),
        ("filter_size_y", 10, "uint32", 0), ("padding_y", 11, "uint32", 0), ("stride_y", 12, "uint32", 0),
        ("output_y", 13, "uint32", 0), ("img_size_y", 14, "uint32", 0), ("dilation", 15, "uint32", 0),
        ("dilation_y", 16, "uint32", 0), ("filter_size_z", 17, "uint32", 0), ("padding_z", 18, "uint32", 0),
        ("stride_z", 19, "uint32", 0), ("output_z", 20, "uint32", 0), ("img_size_z", 21, "uint32", 0)],
    "PoolConfig": [
        ("pool_type", 1, "string", 0), ("channels", 2, "uint32", 0), ("size_x", 3, "uint32", 0),
        ("start", 4, "uint32", 0), ("stride", 5, "uint32", 0), ("output_x", 6, "uint32", 0),
        ("img_size", 7, "uint32", 0), ("padding", 8, "uint32", 0), ("size_y", 9, "uint32", 0),
        ("stride_y", 10, "uint32", 0), ("output_y", 11, "uint32", 0), ("img_size_y", 12, "uint32", 0),
        ("padding_y", 13, "uint32", 0), ("size_z", 14, "uint32", 0), ("stride_z", 15, "uint32", 0),
        ("output_z", 16, "uint32", 0), ("img_size_z", 17, "uint32", 0), ("padding_z", 18, "uint32", 0),
        ("exclude_mode", 19, "bool", 0)],
    "SppConfig": [("image_conf", 1, "ImageConfig", 0), ("pool_type", 2, "string", 0),
                  ("pyramid_height", 3, "uint32", 0)],
    "NormConfig": [
        ("norm_type", 1, "string", 0), ("channels", 2, "uint32", 0), ("size", 3, "uint32", 0),
        ("scale", 4, "double", 0), ("pow", 5, "double", 0), ("output_x", 6, "uint32", 0),
        ("img_size", 7, "uint32", 0), ("blocked", 8, "bool", 0), ("output_y", 9, "uint32", 0),
        ("img_size_y", 10, "uint32", 0)],
    "BlockExpandConfig": [
        ("channels", 1, "uint32", 0), ("stride_x", 2, "uint32", 0), ("stride_y", 3, "uint32", 0),
        ("padding_x", 4, "uint32", 0), ("padding_y", 5, "uint32", 0), ("block_x", 6, "uint32", 0),
        ("block_y", 7, "uint32", 0), ("output_x", 8, "uint32", 0), ("output_y", 9, "uint32", 0),
        ("img_size_x", 10, "uint32", 0), ("img_size_y", 11, "uint32", 0)],
    "MaxOutConfig": [("image_conf", 1, "ImageConfig", 0), ("groups", 2, "uint32", 0)],
    "RowConvConfig": [("context_length", 1, "uint32", 0)],
    "BilinearInterpConfig": [("image_conf", 1, "ImageConfig", 0), ("out_size_x", 2, "uint32", 0),
                             ("out_size_y", 3, "uint32", 0)],
    "PriorBoxConfig": [("min_size", 1, "uint32", 1), ("max_size", 2, "uint32", 1), ("aspect_ratio", 3, "float", 1),
                       ("variance", 4, "float", 1)],
    "PadConfig": [("image_conf", 1, "ImageConfig", 0), ("pad_c", 2, "uint32", 1), ("pad_h", 3, "uint32", 1),
                  ("pad_w", 4, "uint32", 1)],
    "ReshapeConfig": [("height_axis", 1, "uint32", 1), ("width_axis", 2, "uint32", 1)],
    "MultiBoxLossConfig": [
        ("num_classes", 1, "uint32", 0), ("overlap_threshold", 2, "float", 0), ("neg_pos_ratio", 3, "float", 0),
        ("neg_overlap", 4, "float", 0), ("background_id", 5, "uint32", 0), ("input_num", 6, "uint32", 0),
        ("height", 7, "uint32", 0), ("width", 8, "uint32", 0)],
    "DetectionOutputConfig": [
        ("num_classes", 1, "uint32", 0), ("nms_threshold", 2, "float", 0), ("nms_top_k", 3, "uint32", 0),
        ("background_id", 4, "uint32", 0), ("input_num", 5, "uint32", 0), ("keep_top_k", 6, "uint32", 0),
        ("confidence_threshold", 7, "float", 0), ("height", 8, "uint32", 0), ("width", 9, "uint32", 0)],
    "ClipConfig": [("min", 1, "double", 0), ("max", 2, "double", 0)],
    "UpsampleConfig": [
        ("image_conf", 1, "ImageConfig", 0), ("scale", 2, "uint32", 0), ("scale_y", 3, "uint32", 0),
        ("pad_out_x", 4, "bool", 0), ("pad_out_y", 5, "bool", 0), ("upsample_size", 6, "uint32", 0),
        ("upsample_size_y", 7, "uint32", 0)],
    "ROIPoolConfig": [("pooled_width", 1, "uint32", 0), ("pooled_height", 2, "uint32", 0),
                      ("spatial_scale", 3, "float", 0), ("height", 4, "uint32", 0), ("width", 5, "uint32", 0)],
    "ScaleSubRegionConfig": [("image_conf", 1, "ImageConfig", 0), ("value", 2, "float", 0)],
    "ProjectionConfig": [
        ("type", 1, "string", 0), ("name", 2, "string", 0), ("input_size", 3, "uint64", 0),
        ("output_size", 4, "uint64", 0), ("context_start", 5, "int32", 0), ("context_length", 6, "int32", 0),
        ("trainable_padding", 7, "bool", 0), ("conv_conf", 8, "ConvConfig", 0), ("num_filters", 9, "int32", 0),
        ("offset", 11, "uint64", 0), ("pool_conf", 12, "PoolConfig", 0), ("slices", 13, "SliceConfig", 1)],
    "OperatorConfig": [
        ("type", 1, "string", 0), ("input_indices", 2, "int32", 1), ("input_sizes", 3, "uint64", 1),
        ("output_size", 4, "uint64", 0), ("dotmul_scale", 5, "double", 0), ("conv_conf", 6, "ConvConfig", 0),
        ("num_filters", 7, "int32", 0)],
    "LayerInputConfig": [
        ("input_layer_name", 1, "string", 0), ("input_parameter_name", 2, "string", 0),
        ("conv_conf", 3, "ConvConfig", 0), ("pool_conf", 4, "PoolConfig", 0), ("norm_conf", 5, "NormConfig", 0),
        ("proj_conf", 6, "ProjectionConfig", 0), ("block_expand_conf", 7, "BlockExpandConfig", 0),
        ("image_conf", 8, "ImageConfig", 0), ("input_layer_argument", 9, "string", 0),
        ("bilinear_interp_conf", 10, "BilinearInterpConfig", 0), ("maxout_conf", 11, "MaxOutConfig", 0),
        ("spp_conf", 12, "SppConfig", 0), ("priorbox_conf", 13, "PriorBoxConfig", 0), ("pad_conf", 14, "PadConfig", 0),
        ("row_conv_conf", 15, "RowConvConfig", 0), ("multibox_loss_conf", 16, "MultiBoxLossConfig", 0),
        ("detection_output_conf", 17, "DetectionOutputConfig", 0), ("clip_conf", 18, "ClipConfig", 0),
        ("scale_sub_region_conf", 19, "ScaleSubRegionConfig", 0), ("roi_pool_conf", 20, "ROIPoolConfig", 0),
        ("upsample_conf", 21, "UpsampleConfig", 0)],
    "LayerConfig": [
        ("name", 1, "string", 0), ("type", 2, "string", 0), ("size", 3, "uint64", 0),
        ("active_type", 4, "string", 0), ("inputs", 5, "LayerInputConfig", 1),
        ("bias_parameter_name", 6, "string", 0), ("num_filters", 7, "uint32", 0),
        ("shared_biases", 8, "bool", 0), ("partial_sum", 9, "uint32", 0), ("drop_rate", 10, "double", 0),
        ("num_classes", 11, "uint32", 0), ("device", 12, "int32", 0), ("reversed", 13, "bool", 0),
        ("active_gate_type", 14, "string", 0), ("active_state_type", 15, "string", 0),
        ("num_neg_samples", 16, "int32", 0), ("neg_sampling_dist", 17, "double", 1),
        ("output_max_index", 19, "bool", 0), ("softmax_selfnorm_alpha", 21, "double", 0),
        ("directions", 24, "bool", 1), ("norm_by_times", 25, "bool", 0), ("coeff", 26, "double", 0),
        ("average_strategy", 27, "string", 0), ("error_clipping_threshold", 28, "double", 0),
        ("operator_confs", 29, "OperatorConfig", 1), ("NDCG_num", 30, "int32", 0), ("max_sort_size", 31, "int32", 0),
        ("slope", 32, "double", 0), ("intercept", 33, "double", 0),
        ("cos_scale", 34, "double", 0), ("data_norm_strategy", 36, "string", 0), ("bos_id", 37, "uint32", 0),
        ("eos_id", 38, "uint32", 0), ("beam_size", 39, "uint32", 0), ("select_first", 40, "bool", 0),
        ("trans_type", 41, "string", 0), ("selective_fc_pass_generation", 42, "bool", 0),
        ("has_selected_colums", 43, "bool", 0), ("selective_fc_full_mul_ratio", 44, "double", 0),
        ("selective_fc_parallel_plain_mul_thread_num", 45, "uint32", 0),
        ("use_global_stats", 46, "bool", 0), ("moving_average_fraction", 47, "double", 0),
        ("bias_size", 48, "uint32", 0), ("user_arg", 49, "string", 0), ("height", 50, "uint64", 0),
        ("width", 51, "uint64", 0), ("blank", 52, "uint32", 0), ("seq_pool_stride", 53, "int32", 0),
        ("axis", 54, "int32", 0), ("offset", 55, "uint32", 1), ("shape", 56, "uint32", 1),
        ("delta", 57, "double", 0), ("depth", 58, "uint64", 0), ("reshape_conf", 59, "ReshapeConfig", 0),
        ("epsilon", 60, "double", 0), ("factor_size", 61, "uint32", 0)],
    "EvaluatorConfig": [
        ("name", 1, "string", 0), ("type", 2, "string", 0), ("input_layers", 3, "string", 1),
        ("chunk_scheme", 4, "string", 0), ("num_chunk_types", 5, "int32", 0),
        ("classification_threshold", 6, "double", 0), ("positive_label", 7, "int32", 0),
        ("top_k", 13, "int32", 0)],
    "LinkConfig": [("layer_name", 1, "string", 0), ("link_name", 2, "string", 0), ("has_subseq", 3, "bool", 0)],
    "MemoryConfig": [
        ("layer_name", 1, "string", 0), ("link_name", 2, "string", 0), ("boot_layer_name", 3, "string", 0),
        ("boot_bias_parameter_name", 4, "string", 0), ("boot_bias_active_type", 5, "string", 0),
        ("is_sequence", 6, "bool", 0), ("boot_with_const_id", 7, "uint32", 0)],
    "SubModelConfig": [
        ("name", 1, "string", 0), ("layer_names", 2, "string", 1), ("input_layer_names", 3, "string", 1),
        ("output_layer_names", 4, "string", 1), ("evaluator_names", 5, "string", 1),
        ("is_recurrent_layer_group", 6, "bool", 0), ("reversed", 7, "bool", 0),
        ("memories", 8, "MemoryConfig", 1), ("in_links", 9, "LinkConfig", 1), ("out_links", 10, "LinkConfig", 1)],
    "ModelConfig": [
        ("type", 1, "string", 0), ("layers", 2, "LayerConfig", 1), ("parameters", 3, "ParameterConfig", 1),
        ("input_layer_names", 4, "string", 1), ("output_layer_names", 5, "string", 1),
        ("evaluators", 6, "EvaluatorConfig", 1), ("sub_models", 8, "SubModelConfig", 1)],
    "OptimizationConfig": [
        ("batch_size", 3, "int32", 0), ("algorithm", 4, "string", 0),
        ("num_batches_per_send_parameter", 5, "int32", 0), ("num_batches_per_get_parameter", 6, "int32", 0),
        ("learning_rate", 7, "double", 0), ("learning_rate_decay_a", 8, "double", 0),
        ("learning_rate_decay_b", 9, "double", 0), ("l1weight", 10, "double", 0), ("l2weight", 11, "double", 0),
        ("c1", 12, "double", 0), ("backoff", 13, "double", 0), ("owlqn_steps", 14, "int32", 0),
        ("max_backoff", 15, "int32", 0), ("l2weight_zero_iter", 17, "int32", 0),
        ("average_window", 18, "double", 0), ("max_average_window", 19, "int64", 0),
        ("learning_method", 23, "string", 0), ("ada_epsilon", 24, "double", 0),
        ("do_average_in_cpu", 25, "bool", 0), ("ada_rou", 26, "double", 0),
        ("learning_rate_schedule", 27, "string", 0), ("delta_add_rate", 28, "double", 0),
        ("mini_batch_size", 29, "int32", 0), ("use_sparse_remote_updater", 30, "bool", 0),
        ("center_parameter_update_method", 31, "string", 0), ("shrink_parameter_value", 32, "double", 0),
        ("adam_beta1", 33, "double", 0), ("adam_beta2", 34, "double", 0), ("adam_epsilon", 35, "double", 0),
        ("learning_rate_args", 36, "string", 0), ("async_lagged_grad_discard_ratio", 37, "double", 0),
        ("gradient_clipping_threshold", 38, "double", 0)],
    "DataConfig": [
        ("type", 1, "string", 0), ("files", 3, "string", 0), ("async_load_data", 12, "bool", 0),
        ("for_test", 14, "bool", 0), ("load_data_module", 21, "string", 0), ("load_data_object", 22, "string", 0),
        ("load_data_args", 23, "string", 0), ("data_ratio", 25, "int32", 0), ("is_main_data", 26, "bool", 0),
        ("usage_ratio", 27, "double", 0)],
    "TrainerConfig": [
        ("model_config", 1, "ModelConfig", 0), ("data_config", 2, "DataConfig", 0),
        ("opt_config", 3, "OptimizationConfig", 0), ("test_data_config", 4, "DataConfig", 0),
        ("config_files", 5, "string", 1), ("save_dir", 6, "string", 0), ("init_model_path", 7, "string", 0),
        ("start_pass", 8, "int32", 0), ("config_file", 9, "string", 0)],
}
_FIELDS = {m: {f[0]: f for f in fs} for m, fs in _S.items()}
_BYNUM = {m: {f[1]: f for f in fs} for m, fs in _S.items()}
_VARINT = {"int32", "int64", "uint32", "uint64", "bool"}


# ---------------------------------------------------------------- wire codec
def _varint(v):
    v &= (1 << 64) - 1  # negative int32/int64: ten-byte two's complement
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(num, wt):
    return _varint((num << 3) | wt)


def encode(msg, d) -> bytes:
    """Serialise dict ``d`` as message ``msg`` (fields in schema order; repeated
    scalars unpacked, as proto2 does without [packed = true])."""
    out = bytearray()
    for name, num, kind, rep in _S[msg]:
        if name not in d or d[name] is None:
            continue
        vals = d[name] if rep else [d[name]]
        for v in vals:
            if kind in _S:
                b = encode(kind, v)
                out += _key(num, 2) + _varint(len(b)) + b
            elif kind == "string":
                b = v.encode() if isinstance(v, str) else bytes(v)
                out += _key(num, 2) + _varint(len(b)) + b
            elif kind == "double":
                out += _key(num, 1) + struct.pack("<d", float(v))
            elif kind == "float":
                out += _key(num, 5) + struct.pack("<f", float(v))
            else:
                out += _key(num, 0) + _varint(int(v))
    return bytes(out)


def _rvarint(buf, pos):
    r = s = 0
    while True:
        b = buf[pos]
        pos += 1
        r |= (b & 0x7F) << s
        s += 7
        if not b & 0x80:
            return r, pos


def decode(msg, buf: bytes) -> dict:
    d: dict = {}
    pos, n = 0, len(buf)
    while pos < n:
        key, pos = _rvarint(buf, pos)
        num, wt = key >> 3, key & 7
        f = _BYNUM[msg].get(num)
        if wt == 0:
            raw, pos = _rvarint(buf, pos)
        elif wt == 1:
            raw, pos = buf[pos:pos + 8], pos + 8
        elif wt == 5:
            raw, pos = buf[pos:pos + 4], pos + 4
        elif wt == 2:
            ln, pos = _rvarint(buf, pos)
            raw, pos = buf[pos:pos + ln], pos + ln
        else:
            raise ValueError(f"{msg}: unsupported wire type {wt}")
        if f is None:
            continue  # unknown field
        name, _, kind, rep = f
        if kind in _S:
            v = decode(kind, raw)
        elif kind == "string":
            v = raw.decode()
        elif kind == "double":
            v = struct.unpack("<d", raw)[0]
        elif kind == "float":  # the shortest decimal that round-trips in float32 (as text format prints it)
            import numpy as np

            v = float(str(np.float32(struct.unpack("<f", raw)[0])))
        elif wt == 2:  # packed repeated varints
            vals, p = [], 0
            while p < len(raw):
                x, p = _rvarint(raw, p)
                vals.append(x)
            d.setdefault(name, []).extend(vals)
            continue
        elif kind == "bool":
            v = bool(raw)
        elif kind in ("int32", "int64") and raw >= 1 << 63:
            v = raw - (1 << 64)
        else:
            v = raw
        if rep:
            d.setdefault(name, []).append(v)
        else:
            d[name] = v
    return d


# ---------------------------------------------------------------- text format
def _fmt_scalar(kind, v):
    if kind == "string":
        return '"' + v.replace("\\", "\\\\").replace('"', '\\"') + '"'
    if kind == "bool":
        return "true" if v else "false"
    if kind in ("double", "float"):
        r = repr(float(v))
        return r if ("e" in r or "." in r or "inf" in r or "nan" in r) else r + ".0"
    return str(int(v))


def to_text(msg, d, indent=0) -> str:
    pad = "  " * indent
    lines = []
    for name, _, kind, rep in _S[msg]:
        if name not in d or d[name] is None:
            continue
        for v in (d[name] if rep else [d[name]]):
            if kind in _S:
                lines.append(f"{pad}{name} {{")
                lines.append(to_text(kind, v, indent + 1))
                lines.append(f"{pad}}}")
            else:
                lines.append(f"{pad}{name}: {_fmt_scalar(kind, v)}")
    return "\n".join(x for x in lines if x)


_TOK = re.compile(r'\s*(?:(\{)|(\})|("(?:[^"\\]|\\.)*")|([A-Za-z_][\w.\-]*)\s*:|([^\s{}]+))')


def from_text(msg, text, strict=False) -> dict:
    """Parse protobuf text format (as the reference's *.protostr files) into a dict.
    A field the schema does not know is skipped -- or, with ``strict``, kept as
    ``"?<name>": True`` so a comparison against a recorded message reports it."""
    toks = []
    pos = 0
    while pos < len(text):
        m = _TOK.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                break
            raise ValueError(f"text format: cannot parse at {text[pos:pos + 40]!r}")
        pos = m.end()
        toks.append(m.groups())
    i = 0

    def parse(mname):
        nonlocal i
        d = {}
        while i < len(toks):
            ob, cb, st, key, bare = toks[i]
            if cb:
                i += 1
                return d
            if key is None and bare is not None:  # "name {" has no colon
                key = bare
            i += 1
            f = _FIELDS[mname].get(key)
            if f is None and i < len(toks) and toks[i][0]:  # unknown message field: skip its block
                depth = 0
                while True:
                    depth += 1 if toks[i][0] else -1 if toks[i][1] else 0
                    i += 1
                    if depth == 0:
                        break
                if strict:
                    d["?" + key] = True
                continue
            if f is not None and f[2] in _S:
                if toks[i][0]:  # "{"
                    i += 1
                v = parse(f[2])
            else:
                _, _, vs, _, vb = toks[i]
                i += 1
                v = vs if vs is not None else vb
                if f is None:
                    if strict:
                        d["?" + key] = True
                    continue
                kind = f[2]
                if kind == "string":
                    v = bytes(v[1:-1], "utf-8").decode("unicode_escape")
                elif kind == "bool":
                    v = v == "true"
                elif kind in ("double", "float"):
                    v = float(v)
                else:
                    v = int(v)
            if f is None:
                continue
            if f[3]:
                d.setdefault(key, []).append(v)
            else:
                d[key] = v
        return d

    return parse(msg)


# ---------------------------------------------------------------- recording
# default-name prefixes (reference layers.py @wrap_name_default(...); None = the
# function name) and LayerConfig types of the DSL functions
_PREFIX = {
    "mixed_layer": "mixed", "embedding_layer": "embedding", "printer_layer": "print", "priorbox_layer": "priorbox",
    "multibox_loss_layer": "multibox_loss", "detection_output_layer": "detection_output",
    "roi_pool_layer": "roi_pool", "cross_channel_norm_layer": "cross_channel_norm", "pooling_layer": "seq_pooling",
    "lstmemory": "lstmemory", "grumemory": "gru", "seq_reshape_layer": "seqreshape", "img_conv_layer": "conv",
    "img_pool_layer": "pool", "img_pool3d_layer": "pool3d", "upsample_layer": "upsample", "spp_layer": "spp",
    "img_cmrnorm_layer": "crmnorm", "batch_norm_layer": "batch_norm", "addto_layer": "addto",
    "concat_layer": "concat", "seq_concat_layer": "seqconcat", "lstm_step_layer": "lstm_step",
    "gru_step_layer": "gru_step", "gru_step_naive_layer": "gru_step_naive", "recurrent_group": "recurrent_group",
    "classification_cost": "cost", "pad_layer": "pad", "dropout_layer": "dropout", "switch_order_layer": "switch_order",
    "clip_layer": "clip", "img_conv3d_layer": "conv3d", "scale_shift_layer": "scale_shift", "resize_layer": "resize",
    "sub_seq_layer": "sub_seq", "scale_sub_region_layer": "scale_sub_region",
}
_TYPE = {
    "data_layer": "data", "fc_layer": "fc", "printer_layer": "print", "priorbox_layer": "priorbox",
    "multibox_loss_layer": "multibox_loss", "detection_output_layer": "detection_output", "roi_pool_layer": "roi_pool",
    "cross_channel_norm_layer": "norm", "lstmemory": "lstmemory", "grumemory": "gated_recurrent",
    "last_seq": "seqlastins", "first_seq": "seqlastins", "expand_layer": "expand", "repeat_layer": "featmap_expand",
    "seq_reshape_layer": "seqreshape", "interpolation_layer": "interpolation", "bilinear_interp_layer": "bilinear_interp",
    "power_layer": "power", "scaling_layer": "scaling", "trans_layer": "trans", "rotate_layer": "rotate",
    "cos_sim": "cos", "l2_distance_layer": "l2_distance", "hsigmoid": "hsigmoid", "img_conv_layer": "exconv",
    "img_pool_layer": "pool", "img_pool3d_layer": "pool3d", "upsample_layer": "upsample", "spp_layer": "spp",
    "img_cmrnorm_layer": "norm", "batch_norm_layer": "batch_norm", "sum_to_one_norm_layer": "sum_to_one_norm",
    "row_l2_norm_layer": "row_l2_norm", "addto_layer": "addto", "concat_layer": "concat",
    "seq_concat_layer": "seqconcat", "lstm_step_layer": "lstm_step", "gru_step_layer": "gru_step",
    "get_output_layer": "get_output", "recurrent_layer": "recurrent", "maxid_layer": "maxid",
    "dot_prod_layer": "dot_prod", "out_prod_layer": "out_prod", "eos_layer": "eos_id", "square_error_cost": "square_error",
    "regression_cost": "square_error", "mse_cost": "square_error", "classification_cost": "multi-class-cross-entropy",
    "pad_layer": "pad", "conv_shift_layer": "conv_shift", "tensor_layer": "tensor", "selective_fc_layer": "selective_fc",
    "sampling_id_layer": "sampling_id", "slope_intercept_layer": "slope_intercept", "linear_comb_layer": "convex_comb",
    "block_expand_layer": "blockexpand", "maxout_layer": "maxout", "ctc_layer": "ctc", "warp_ctc_layer": "warp_ctc",
    "crf_layer": "crf", "crf_decoding_layer": "crf_decoding", "nce_layer": "nce", "rank_cost": "rank-cost",
    "lambda_cost": "lambda_cost", "cross_entropy": "multi-class-cross-entropy",
    "cross_entropy_with_selfnorm": "multi_class_cross_entropy_with_selfnorm", "sum_cost": "sum_cost",
    "huber_regression_cost": "huber_regression", "huber_classification_cost": "huber_classification",
    "multi_binary_label_cross_entropy": "multi_binary_label_cross_entropy",
    "cross_entropy_over_beam": "cross_entropy_over_beam", "smooth_l1_cost": "smooth_l1",
    "multiplex_layer": "multiplex", "row_conv_layer": "row_conv", "prelu_layer": "prelu",
    "switch_order_layer": "switch_order", "crop_layer": "crop", "sub_nested_seq_layer": "sub_nested_seq",
    "clip_layer": "clip", "seq_slice_layer": "seq_slice", "kmax_seq_score_layer": "kmax_seq_score",
    "img_conv3d_layer": "conv3d", "scale_shift_layer": "scale_shift", "resize_layer": "resize",
    "sub_seq_layer": "subseq", "scale_sub_region_layer": "scale_sub_region",
    "factorization_machine": "factorization_machine", "pooling_layer": "max", "mixed_layer": "mixed",
    "embedding_layer": "mixed", "dropout_layer": "addto", "memory": "agent",
    "recurrent_group": "recurrent_layer_group",
}
_ACT = {None: "", "linear": "", "identity": "", "exp": "exponential", "soft_relu": "softrelu"}
# layers whose size is their input's (the reference sets size = input.size)
_SAME_SIZE = {"trans_layer", "first_seq", "last_seq", "dropout_layer", "batch_norm_layer", "clip_layer",
              "row_l2_norm_layer", "sum_to_one_norm_layer", "scaling_layer", "slope_intercept_layer",
              "power_layer", "rotate_layer", "prelu_layer", "pooling_layer", "addto_layer", "expand_layer",
              "img_cmrnorm_layer", "crf_layer"}
# projections without a parameter (they take no weight of the mixed layer's)
_PARAMLESS = {"identity", "identity_offset", "slice"}
# functions that are not layers (projections / operators feed mixed / concat layers)
_NOT_LAYERS = {"settings", "outputs", "get_config_arg", "define_py_data_sources2", "parse_config"}


class Recorder:
    """Per-parse state: LayerConfigs, ParameterConfigs and the variable -> layer map."""

    def __init__(self):
        self.layers = []
        self.params = []
        self.param_map = {}  # v1 parameter name -> Fluid parameter name
        self.of_var = {}      # id(fluid Variable) -> layer name
        self.vars = []        # keeps the recorded Variables alive (ids stay unique)
        self.count = {}
        self.inputs = []
        self.outputs = []
        self.depth = 0
        self.by_name = {}     # layer name -> its LayerConfig (image dims of inputs)
        self.evaluators = []  # EvaluatorConfigs (classification_cost's default evaluator)
        self.parents = {}     # layer name -> parent layer names (networks.outputs DFS)
        self.groups = []      # open recurrent_group records (innermost last)
        self.sub_models = []  # finished recurrent_group SubModelConfigs
        self.inner = set()    # layer names that belong to a recurrent group

    def name_for(self, fn, given):
        if given:
            return given
        pre = _PREFIX.get(fn, fn)
        i = self.count.get(pre, 0)
        self.count[pre] = i + 1
        return f"__{pre}_{i}__"

    def layer_name(self, v):
        return self.of_var.get(id(v))


_REC: list = []


def start():
    _REC[:] = [Recorder()]
    return _REC[0]


def current():
    return _REC[0] if _REC else None


def _vsize(v):
    s = getattr(v, "v2_size", None)
    if s is None:
        sh = getattr(v, "shape", None)
        if sh and len(sh) >= 4:  # an image [N, C, H, W]: the layer size is C * H * W
            s = _prod(sh[1:])
        else:
            s = int(sh[-1]) if sh else None
    return s


def _is_var(x):
    return hasattr(x, "block") and hasattr(x, "name") and hasattr(x, "shape")


def _flat_inputs(fn, args, kw):
    """Layer inputs in signature order: Variables and projections (with .input)."""
    try:
        ba = inspect.signature(fn).bind_partial(*args, **kw)
        items = [(k, v) for k, v in ba.arguments.items() if k not in ("name", "act", "size", "param_attr",
                                                                       "bias_attr", "layer_attr")]
    except (TypeError, ValueError):
        items = [(None, a) for a in args] + list(kw.items())
    out, later = [], []
    for _, v in items:
        if isinstance(v, dict):  # **kw of the DSL function (e.g. a cost's weight layer)
            v = [w for k, w in v.items() if k not in ("name", "act", "size", "param_attr", "bias_attr", "layer_attr")]
        for x in (v if isinstance(v, (list, tuple)) else [v]):
            if _is_var(x):
                out.append((x, None))
            elif getattr(x, "v1_operands", None):
                # an operator (config_parser.py MixedLayer): its first operand takes the
                # operator's place among the inputs, the others follow all the inputs
                out.append((x.v1_operands[0], x))
                later.extend((o, x) for o in x.v1_operands[1:])
            elif _is_var(getattr(x, "input", None)):
                out.append((x.input, x))  # a projection / operator
    return out + later


def _attr_name(attr, i):
    """The user-given parameter name of input i's ParamAttr (a list holds one per input)."""
    if isinstance(attr, (list, tuple)):
        attr = attr[i] if i < len(attr) else None
    if attr is None or isinstance(attr, bool):
        return None
    return getattr(attr, "name", None)


def _apply_pattr(prec, attr):
    """ParameterAttribute semantics (reference attrs.py): initial_max / min -> uniform
    (strategy 1, mean / std the interval's centre / half width); an explicit mean or
    std -> normal with those; either way no smart init.  learning_rate, l2_rate
    (decay_rate) and is_static carried over."""
    if attr is None or isinstance(attr, bool):
        return
    mx, mn = getattr(attr, "initial_max", None), getattr(attr, "initial_min", None)
    std, mean = getattr(attr, "initial_std", None), getattr(attr, "initial_mean", None)
    if mx is not None or mn is not None:
        mx, mn = float(mx if mx is not None else 0.0), float(mn if mn is not None else 0.0)
        prec.update(initial_mean=(mx + mn) / 2, initial_std=(mx - mn) / 2, initial_strategy=1, initial_smart=False)
    elif std is not None or mean is not None:
        prec.update(initial_mean=float(mean or 0.0), initial_std=float(std if std is not None else 0.01),
                    initial_strategy=0, initial_smart=False)
    if getattr(attr, "learning_rate", None) is not None:
        prec["learning_rate"] = float(attr.learning_rate)
    if getattr(attr, "l2_rate", None) is not None:
        prec["decay_rate"] = float(attr.l2_rate)
    if getattr(attr, "is_static", False):
        prec["is_static"] = True


def _pattr(attr, i):
    if isinstance(attr, (list, tuple)):
        return attr[i] if i < len(attr) else None
    return attr


def _param_dims(p):
    d = [int(v) for v in p.shape]
    return [1] + d if len(d) == 1 else d  # a vector weight (dot_mul / scaling) is [1, n]


def unwrap(x):
    """A finished ``with mixed_layer(...) as m`` context stands for its layer."""
    if type(x).__name__ == "_MixedCtx":
        return x.m.out
    if isinstance(x, list):
        return [unwrap(v) for v in x]
    if isinstance(x, tuple):
        return tuple(unwrap(v) for v in x)
    return x


def recorded(fn_name, fn):
    """Wrap a DSL layer function so a call at config level records its LayerConfig."""

    def wrapper(*args, **kw):
        args = tuple(unwrap(a) for a in args)
        kw = {k: unwrap(v) for k, v in kw.items()}
        rec = current()
        if rec is None or rec.depth:
            return fn(*args, **kw)
        from ..v2._core import STATE

        if fn_name == "recurrent_group":
            return _record_group(rec, fn, args, kw)
        if fn_name == "memory" and rec.groups:
            return _record_memory(rec, fn, args, kw)
        blk = STATE["main"].global_block()
        before = {p.name for p in blk.all_parameters()}
        rec.depth += 1
        try:
            out = fn(*args, **kw)
        finally:
            rec.depth -= 1
        if type(out).__name__ == "_MixedCtx":
            # ``with mixed_layer(...) as m: m += ...``: recorded when the block exits
            out.m.on_finish = lambda m, _a=args, _k=kw: _record(rec, fn_name, fn, _a, dict(_k, input=list(m.terms)),
                                                                 m.out, before, blk)
            return out
        return _record(rec, fn_name, fn, args, kw, out, before, blk)

    wrapper.__name__ = fn.__name__
    wrapper.__doc__ = fn.__doc__
    wrapper.__wrapped__ = fn
    return wrapper


def _record(rec, fn_name, fn, args, kw, out, before, blk):
    """The LayerConfig (and ParameterConfigs) of one finished layer call."""
    if True:
        new = [p for p in blk.all_parameters() if p.name not in before]
        outs = out if isinstance(out, (list, tuple)) else [out]
        if not outs or not _is_var(outs[0]):
            return out
        v = outs[0]
        name = rec.name_for(fn_name, kw.get("name") if fn_name != "data_layer" else (kw.get("name") or args[0]))
        base = name  # projection names inside a recurrent group keep the unsuffixed layer name
        if rec.groups:
            name = f"{base}@{rec.groups[-1]['name']}"
            rec.groups[-1]["layer_names"].append(name)
            rec.inner.add(name)
        ins = _flat_inputs(fn, args, kw)
        typ = _TYPE.get(fn_name, fn_name.replace("_layer", ""))
        act = kw.get("act")
        from ..v2.activation import act_name

        an = act_name(act) if act is not None else ("tanh" if fn_name in ("fc_layer", "selective_fc_layer") else None)
        size = kw.get("size") if isinstance(kw.get("size"), int) else None
        if fn_name == "data_layer":
            size = kw.get("size", args[1] if len(args) > 1 else None)
        if fn_name in _SAME_SIZE and ins:
            size = _vsize(ins[0][0])
        if fn_name == "concat_layer":
            size = sum(_vsize(x) or 0 for x, _ in ins)
        if size is None:
            size = _vsize(v)
        lc = {"name": name, "type": typ, "size": size, "active_type": _ACT.get(an, an or "")}
        by_pname = {p.name: p for p in blk.all_parameters()}
        weights = [p for p in new if (len(p.shape) >= 2 or getattr(p, "_v1_weight", False))
                   and not getattr(p, "_v1_bias", False)]
        wn = {p.name for p in weights}
        biases = [p for p in new if p.name not in wn]
        layer_inputs = []
        projs = any(pr is not None for _, pr in ins)
        # user-named weights: the layer's param_attr (one per input when a list), else a
        # projection's own; they are not handed out by position
        unames = []
        for i, (x, pr) in enumerate(ins):
            un = _attr_name(kw.get("param_attr"), i)
            if un is None and pr is not None:
                un = _attr_name(getattr(pr, "v1_param_attr", None), 0)
            unames.append(un)
        weights = [p for p in weights if p.name not in set(unames)]
        wi = 0
        if fn_name == "concat_layer" and projs:
            lc["type"] = "concat2"
        for i, (x, pr) in enumerate(ins):
            li = {"input_layer_name": rec.layer_name(x) or x.name}
            if pr is not None and fn_name == "concat_layer":
                li["proj_conf"] = {"type": getattr(pr, "v1_type", "identity"), "name": f"_{base}.w{i}",
                                   "input_size": _vsize(x), "output_size": _vsize(x)}
            if (pr is not None and fn_name in ("mixed_layer", "embedding_layer") and getattr(pr, "v1_type", None)
                    and not getattr(pr, "v1_operands", None)):
                li["proj_conf"] = {"type": _PROJ_TYPE.get(pr.v1_type, pr.v1_type), "name": f"_{base}.w{i}",
                                   "input_size": _vsize(x), "output_size": size}
            uname = unames[i]
            if uname is not None and uname in by_pname:  # ParamAttr(name=...): a named, possibly shared, weight
                li["input_parameter_name"] = uname
                if uname not in rec.param_map:
                    rec.param_map[uname] = uname
                    dims = _param_dims(by_pname[uname])
                    rec.params.append({"name": uname, "size": int(_prod(dims)), "initial_mean": 0.0,
                                       "initial_std": 1.0 / max(dims[0], 1) ** 0.5, "dims": dims,
                                       "initial_strategy": 0, "initial_smart": True})
                    _apply_pattr(rec.params[-1], _pattr(kw.get("param_attr"), i) if pr is None or
                             getattr(pr, "v1_param_attr", None) is None else pr.v1_param_attr)
            elif wi < len(weights) and (pr is None or (getattr(pr, "v1_type", None) not in _PARAMLESS
                                                      and not getattr(pr, "v1_operands", None))):
                pname = f"_{name}.w{i}"
                li["input_parameter_name"] = pname
                rec.param_map[pname] = weights[wi].name
                dims = _param_dims(weights[wi])
                if pr is not None and getattr(pr, "v1_type", None) == "fc" and size and _vsize(x):
                    dims = [int(_vsize(x)), int(size)]  # v1: [input width, layer width] whatever the id layout
                wi += 1
                rec.params.append({"name": pname, "size": int(_prod(dims)), "initial_mean": 0.0,
                                   "initial_std": 1.0 / max(dims[0], 1) ** 0.5, "dims": dims,
                                   "initial_strategy": 0, "initial_smart": True})
                _apply_pattr(rec.params[-1], _pattr(kw.get("param_attr"), i))
            layer_inputs.append(li)
        if layer_inputs:
            lc["inputs"] = layer_inputs
        bname = _attr_name(kw.get("bias_attr"), 0)
        if bname is not None and bname in by_pname:
            lc["bias_parameter_name"] = bname
            if bname not in rec.param_map:
                rec.param_map[bname] = bname
                n = int(_prod(_param_dims(by_pname[bname])))
                rec.params.append({"name": bname, "size": n, "initial_mean": 0.0, "initial_std": 0.0,
                                   "dims": [1, n], "initial_strategy": 0, "initial_smart": False})
                _apply_pattr(rec.params[-1], kw.get("bias_attr"))
        elif biases:
            pname = f"_{name}.wbias"
            lc["bias_parameter_name"] = pname
            rec.param_map[pname] = biases[0].name
            n = int(_prod(_param_dims(biases[0])))
            rec.params.append({"name": pname, "size": n, "initial_mean": 0.0, "initial_std": 0.0, "dims": [1, n],
                               "initial_strategy": 0, "initial_smart": False})
            _apply_pattr(rec.params[-1], kw.get("bias_attr"))
        if fn_name == "data_layer":
            rec.inputs.append(name)
        # LayerOutput.parents of the reference helpers: the layer inputs, except for
        # layers whose index / range inputs are not graph parents
        pnames = [rec.layer_name(x) for x, _ in ins if rec.layer_name(x)]
        rec.parents[name] = pnames[:1] if fn_name in _FIRST_PARENT_ONLY else pnames
        la = kw.get("layer_attr")
        if la is not None:
            if getattr(la, "drop_rate", None):
                lc["drop_rate"] = float(la.drop_rate)
            if getattr(la, "error_clipping_threshold", None):
                lc["error_clipping_threshold"] = float(la.error_clipping_threshold)
        extra = _EXTRA.get(fn_name)
        if extra is not None:
            extra(lc, args, kw, ins, rec, name)
        rec.layers.append(lc)
        rec.by_name[name] = lc
        rec.of_var[id(v)] = name
        rec.vars.append(v)
        return out


def _add_layer(rec, lc, var=None, parents=()):
    rec.layers.append(lc)
    rec.by_name[lc["name"]] = lc
    rec.parents[lc["name"]] = list(parents)
    if var is not None:
        rec.of_var[id(var)] = lc["name"]
        rec.vars.append(var)


def _record_memory(rec, fn, args, kw):
    """memory() inside a recurrent group (config_parser.py Memory / RecurrentLayerGroup):
    an ``agent`` layer ``<name>+delay1@<group>`` (``__memory_<k>__@<group>`` when
    anonymous, k counting every memory() call), linked to the group's layer of that
    name in the group's ``memories``."""
    g = rec.groups[-1]
    name = _arg(args, kw, "name", 0)
    size = _arg(args, kw, "size", 1)
    boot = _arg(args, kw, "boot_layer", 3)
    k = rec.count.get("memory", 0)
    rec.count["memory"] = k + 1
    agent = f"{name}+delay1@{g['name']}" if name else f"__memory_{k}__@{g['name']}"
    out = fn(*args, **kw)
    _add_layer(rec, {"name": agent, "type": "agent", "size": size, "active_type": ""}, out)
    g["layer_names"].append(agent)
    rec.inner.add(agent)
    ent = {"layer_name": f"{name}@{g['name']}" if name else None, "link_name": agent}
    if boot is not None and rec.layer_name(boot):
        ent["boot_layer_name"] = rec.layer_name(boot)
    g["memories"].append(ent)
    if not name and hasattr(out, "set_input"):
        bind = out.set_input

        def set_input(layer, _b=bind, _e=ent):
            _b(layer)
            _e["layer_name"] = rec.layer_name(layer)
        out.set_input = set_input
    return out


def _record_group(rec, fn, args, kw):
    """recurrent_group (config_parser.py RecurrentLayerGroupBegin / End): a
    ``recurrent_layer_group`` layer, one ``scatter_agent`` per sequence input
    (``<input>@<group>``), the step's layers named ``<layer>@<group>``, one
    ``gather_agent`` per step output under the output's own name, and a
    SubModelConfig with the memories and in / out links."""
    from .layers_v1 import StaticInput, SubsequenceInput

    step = _arg(args, kw, "step", 0)
    inp = _arg(args, kw, "input", 1)
    reverse = bool(_arg(args, kw, "reverse", 2, False))
    gname = rec.name_for("recurrent_group", _arg(args, kw, "name", 3))
    _add_layer(rec, {"name": gname, "type": "recurrent_layer_group", "active_type": ""})
    g = {"name": gname, "layer_names": [], "is_recurrent_layer_group": True, "reversed": reverse, "memories": [],
         "in_links": [], "out_links": [], "_outs": []}
    ins = list(inp) if isinstance(inp, (list, tuple)) else [inp]

    def step_rec(*sargs):
        for x, a in zip(ins, sargs):
            if isinstance(x, StaticInput):
                continue
            outer = x.input if isinstance(x, SubsequenceInput) else x
            on = rec.layer_name(outer) or outer.name
            agent = f"{on}@{gname}"
            _add_layer(rec, {"name": agent, "type": "scatter_agent", "size": _vsize(outer), "active_type": ""}, a,
                       [on])
            g["layer_names"].append(agent)
            rec.inner.add(agent)
            g["in_links"].append({"layer_name": on, "link_name": agent})
        res = step(*sargs)
        g["_outs"] = list(res) if isinstance(res, (list, tuple)) else [res]
        return res

    a2, kw2 = list(args), dict(kw)
    if "step" in kw2:
        kw2["step"] = step_rec
    else:
        a2[0] = step_rec
    rec.groups.append(g)
    try:
        out = fn(*a2, **kw2)
    finally:
        rec.groups.pop()
    outs = list(out) if isinstance(out, (list, tuple)) else [out]
    for inner, o in zip(g["_outs"], outs):
        iname = rec.layer_name(inner)
        if not iname:
            continue
        gather = iname.rsplit("@", 1)[0]
        _add_layer(rec, {"name": gather, "type": "gather_agent", "size": _vsize(inner), "active_type": ""}, o,
                   [iname])
        g["out_links"].append({"layer_name": iname, "link_name": gather})
    rec.sub_models.append(g)
    return out


# ---------------------------------------------------------------- per-type fields
# The LayerConfig fields beyond name / type / size / activation / inputs that the
# reference parser sets for a layer type (its Layer classes in
# trainer/config_parser.py), derived here from the DSL call's arguments.
def _arg(fn_args, kw, name, pos, default=None):
    if name in kw:
        return kw[name]
    return fn_args[pos] if len(fn_args) > pos else default


def _level(v, default="non-seq"):
    return v if isinstance(v, str) else default


def _in_lc(rec, ins, i=0):
    if len(ins) <= i:
        return {}
    return rec.by_name.get(rec.layer_name(ins[i][0]) or "", {})


def _hwd_from(lc, src):
    """set_layer_height_width + set_layer_depth from an input layer (unset: 0, 0, 1)."""
    lc["height"] = int(src.get("height", 0))
    lc["width"] = int(src.get("width", 0))
    lc["depth"] = int(src.get("depth", 1))


# ---- image geometry (reference config_parser.py get_img_size / cnn_output_size /
# parse_conv / parse_pool / parse_norm / parse_image, re-derived from the layer
# records: an input layer's size, height, width, depth and its output channels,
# kept as the private "_num_filters" key -- LayerOutput.num_filters)
def _xy(kw, key, default):
    """A DSL size argument that may be an (x, y[, z]) sequence; key_y overrides y."""
    v = kw.get(key, default)
    if isinstance(v, (list, tuple)):
        x, y = int(v[0]), int(v[1])
    else:
        x = y = int(v)
    if kw.get(key + "_y") is not None:
        y = int(kw[key + "_y"])
    return x, y


def _z(kw, key, default_x):
    v = kw.get(key)
    if isinstance(v, (list, tuple)) and len(v) > 2:
        return int(v[2])
    if kw.get(key + "_z") is not None:
        return int(kw[key + "_z"])
    return default_x


def _out_size(img, k, pad, stride, caffe, dil=1):
    import math

    fs = (k - 1) * dil + 1
    o = (2 * pad + img - fs) / float(stride)
    return 1 + int(math.floor(o) if caffe else math.ceil(o))


def _img_size(k, out, pad, stride, caffe, dil=1):
    fs = (k - 1) * dil + 1
    v = (out - 1) * stride + fs - 2 * pad
    return v if caffe else v + 1


def _channels(kw, rec, ins, key="num_channels"):
    c = kw.get(key)
    if c:
        return int(c)
    src = _in_lc(rec, ins)
    if src.get("_num_filters"):
        return int(src["_num_filters"])
    hwd = int(src.get("height") or 0) * int(src.get("width") or 0) * int(src.get("depth") or 1)
    if hwd and src.get("size"):
        return int(src["size"]) // hwd
    sh = list(getattr(ins[0][0], "shape", []) or []) if ins else []
    return int(sh[1]) if len(sh) >= 4 else int(src.get("size") or _vsize(ins[0][0]) or 1)


def _img_wh(rec, ins, c):
    src = _in_lc(rec, ins)
    size = int(src.get("size") or _vsize(ins[0][0]) or 0)
    pix = size // max(c, 1)
    w = int(src.get("width") or 0) or int(pix ** 0.5)
    h = int(src.get("height") or 0) or (pix // w if w else 0)
    return w, h


def _img_whd(rec, ins):
    src = _in_lc(rec, ins)
    return int(src.get("width") or 0), int(src.get("height") or 0), int(src.get("depth") or 1)


def _image_conf(rec, ins, c, three_d=False):
    if three_d:
        w, h, d = _img_whd(rec, ins)
        return {"channels": c, "img_size": w, "img_size_y": h, "img_size_z": d}
    w, h = _img_wh(rec, ins, c)
    return {"channels": c, "img_size": w, "img_size_y": h}


def _pool_type(pt, default="max"):
    kind = type(pt).__name__ if pt is not None else default
    return "avg-projection" if kind.startswith(("Avg", "CudnnAvg")) else "max-projection"


def _x_data(lc, a, kw, ins, rec, name):
    h, w, d = kw.get("height"), kw.get("width"), kw.get("depth")
    if h and w:
        lc["height"], lc["width"] = int(h), int(w)
    if d:
        lc["depth"] = int(d)


def _x_addto(lc, a, kw, ins, rec, name):
    src = _in_lc(rec, ins)
    for i in range(len(ins)):
        c = _in_lc(rec, ins, i)
        if c.get("height"):
            src = c
    _hwd_from(lc, src)


def _x_concat(lc, a, kw, ins, rec, name):
    if lc.get("type") == "concat":
        _hwd_from(lc, _in_lc(rec, ins))


def _x_seqins(first):
    def f(lc, a, kw, ins, rec, name):
        lc["trans_type"] = _level(kw.get("agg_level"))
        lc["seq_pool_stride"] = int(kw.get("stride", -1))
        if first:
            lc["select_first"] = True
    return f


def _x_expand(lc, a, kw, ins, rec, name):
    lc["trans_type"] = _level(kw.get("expand_level"))


def _x_repeat(lc, a, kw, ins, rec, name):
    lc["num_filters"] = int(_arg(a, kw, "num_repeats", 1))
    if not kw.get("as_row_vector", True):
        lc["user_arg"] = "as_col_vec"


def _act_or(kw, key, default):
    from ..v2.activation import act_name

    v = kw.get(key)
    an = act_name(v) if v is not None else default
    return _ACT.get(an, an)


def _set_params(rec, name, lc, specs):
    """Replace the layer's recorded parameters by the reference's (name, dims, std)."""
    rec.params[:] = [p for p in rec.params if not p["name"].startswith(f"_{name}.")]
    for pname, dims, std, smart in specs:
        rec.params.append({"name": pname, "size": int(_prod(dims)), "initial_mean": 0.0, "initial_std": std,
                           "dims": list(dims), "initial_strategy": 0, "initial_smart": smart})


def _x_lstm(lc, a, kw, ins, rec, name):
    size = int(lc.get("size") or 0) or (_vsize(ins[0][0]) or 0) // 4
    lc["size"] = size
    lc["reversed"] = bool(kw.get("reverse", False))
    lc["active_type"] = _act_or(kw, "act", "tanh")
    lc["active_gate_type"] = _act_or(kw, "gate_act", "sigmoid")
    lc["active_state_type"] = _act_or(kw, "state_act", "tanh")
    lc["bias_parameter_name"] = f"_{name}.wbias"
    _set_params(rec, name, lc, [(f"_{name}.w0", [size, size, 4], 1.0 / size ** 0.5, True),
                                (f"_{name}.wbias", [1, 7 * size], 0.0, False)])


def _x_gru(lc, a, kw, ins, rec, name):
    size = int(lc.get("size") or 0) or (_vsize(ins[0][0]) or 0) // 3
    lc["size"] = size
    lc["reversed"] = bool(kw.get("reverse", False))
    lc["active_type"] = _act_or(kw, "act", "tanh")
    lc["active_gate_type"] = _act_or(kw, "gate_act", "sigmoid")
    lc["bias_parameter_name"] = f"_{name}.wbias"
    _set_params(rec, name, lc, [(f"_{name}.w0", [size, 3 * size], 1.0 / size ** 0.5, True),
                                (f"_{name}.wbias", [1, 3 * size], 0.0, False)])


def _x_hsigmoid(lc, a, kw, ins, rec, name):
    nc = int(kw.get("num_classes") or 2)
    lc["num_classes"] = nc
    lc["size"] = 1
    for li in lc.get("inputs", [])[1:]:
        li.pop("input_parameter_name", None)
    lc["bias_parameter_name"] = f"_{name}.wbias"
    insz = _vsize(ins[0][0]) or 0
    # smart initialisation: std = 1 / sqrt(dims[0])
    _set_params(rec, name, lc, [(f"_{name}.w0", [nc - 1, insz], 1.0 / (nc - 1) ** 0.5, True),
                                (f"_{name}.wbias", [1, nc - 1], 0.0, False)])


def _x_selective_fc(lc, a, kw, ins, rec, name):
    lc["selective_fc_pass_generation"] = bool(kw.get("pass_generation", False))
    lc["has_selected_colums"] = bool(kw.get("has_selected_colums", True))
    lc["selective_fc_full_mul_ratio"] = float(kw.get("mul_ratio", 0.02))
    for p in rec.params:
        if p["name"] == f"_{name}.w0":
            p["is_sparse"] = False


_FIRST_PARENT_ONLY = {"seq_slice_layer", "sub_nested_seq_layer"}
_PROJ_TYPE = {"identity_offset": "identity_offset", "trans_fc": "trans_fc"}


def _x_weight_first(lc, a, kw, ins, rec, name):
    """scaling / interpolation / power layers list the weight layer first."""
    n = len(lc.get("inputs", []))
    if n >= 2:  # the weight is the last argument of the DSL call
        lc["inputs"] = lc["inputs"][-1:] + lc["inputs"][:-1]
        ps = rec.parents.get(name, [])
        rec.parents[name] = ps[-1:] + ps[:-1]


def _x_cos(lc, a, kw, ins, rec, name):
    """cos_sim: a vector against a matrix of `size` rows is the "cos_vm" layer."""
    size = int(kw.get("size", 1) or 1)
    lc["size"] = size
    if size > 1:
        lc["type"] = "cos_vm"
    lc["cos_scale"] = float(kw.get("scale", 1.0))


def _x_reorder(order, size=None):
    """Layers whose LayerConfig lists the inputs in another order than the DSL call
    (detection_output: priorbox, loc, conf; multibox_loss: priorbox, label, loc, conf)."""
    def f(lc, a, kw, ins, rec, name):
        by = {k: i for i, k in enumerate(("input_loc", "input_conf", "priorbox", "label"))}
        li = lc.get("inputs", [])
        lc["inputs"] = [li[by[k]] for k in order if by[k] < len(li)]
        rec.parents[name] = [x["input_layer_name"] for x in lc["inputs"]]
        if size is not None:
            lc["size"] = size(kw)
    return f


def _x_beam(lc, a, kw, ins, rec, name):
    """cross_entropy_over_beam: (scores, selected candidates, gold) of every beam."""
    beams = kw.get("input") if "input" in kw else (a[0] if a else [])
    beams = beams if isinstance(beams, (list, tuple)) else [beams]
    ls = []
    for b in beams:
        for v in (b.candidate_scores, b.selected_candidates, b.gold):
            ls.append({"input_layer_name": rec.layer_name(v) or v.name})
    lc["inputs"] = ls
    rec.parents[name] = [x["input_layer_name"] for x in ls]
    lc.pop("size", None)


def _x_no_size(lc, a, kw, ins, rec, name):
    lc.pop("size", None)  # the reference leaves this cost's size unset


def _x_tensor(lc, a, kw, ins, rec, name):
    """TensorLayer: one [a, b, size] weight on the first input, a [1, size] bias."""
    size = int(lc["size"])
    da, db = _vsize(ins[0][0]) or 0, _vsize(ins[1][0]) or 0
    fl = rec.param_map.pop(f"_{name}.w1", None)
    if fl is not None:
        rec.param_map[f"_{name}.wbias"] = fl
    for li in lc.get("inputs", [])[1:]:
        li.pop("input_parameter_name", None)
    lc["bias_parameter_name"] = f"_{name}.wbias"
    _set_params(rec, name, lc, [(f"_{name}.w0", [da, db, size], 1.0 / max(da, 1) ** 0.5, True),
                                (f"_{name}.wbias", [1, size], 0.0, False)])


def _x_ctc(lc, a, kw, ins, rec, name):
    """CTC costs: size = number of classes incl. the blank = label size + 1."""
    size = kw.get("size")
    lc["size"] = int(size) if size else (_vsize(ins[1][0]) or 0) + 1
    lc["norm_by_times"] = bool(kw.get("norm_by_times", False))
    if "blank" in kw:
        lc["blank"] = int(kw["blank"])


def _x_slope(lc, a, kw, ins, rec, name):
    lc["slope"] = kw.get("slope", 1.0)
    lc["intercept"] = kw.get("intercept", 0.0)


def _x_factor(lc, a, kw, ins, rec, name):
    lc["factor_size"] = int(_arg(a, kw, "factor_size", 1))


def _x_coeff(lc, a, kw, ins, rec, name):
    lc["coeff"] = float(kw.get("coeff", 1.0))


def _x_kmax(lc, a, kw, ins, rec, name):
    lc.pop("size", None)
    lc["beam_size"] = int(kw.get("beam_size", 1))


def _x_same_size(lc, a, kw, ins, rec, name):
    lc["size"] = _vsize(ins[0][0]) if ins else lc.get("size")


def _x_scale_shift(lc, a, kw, ins, rec, name):
    # one scalar scale w0 (+ scalar bias unless bias_attr=False)
    has_b = kw.get("bias_attr", None) is not False
    lc["inputs"] = [{"input_layer_name": rec.layer_name(ins[0][0]) or ins[0][0].name,
                     "input_parameter_name": f"_{name}.w0"}]
    specs = [(f"_{name}.w0", [1, 1], 1.0, True)]
    if has_b:
        lc["bias_parameter_name"] = f"_{name}.wbias"
        specs.append((f"_{name}.wbias", [1, 1], 0.0, False))
    else:
        lc.pop("bias_parameter_name", None)
    _set_params(rec, name, lc, specs)


def _x_seq_slice(lc, a, kw, ins, rec, name):
    if kw.get("ends", 1) is None:
        lc["select_first"] = True
    elif kw.get("starts", 1) is None:
        lc["select_first"] = False


def _x_pooling(lc, a, kw, ins, rec, name):
    """pooling_layer: MaxLayer ("max") or AverageLayer ("average" + strategy)."""
    pt = kw.get("pooling_type")
    kind = type(pt).__name__ if pt is not None else "Max"
    if kind in ("Max", "MaxPooling"):
        lc["type"] = "max"
        if getattr(pt, "output_max_index", None) is not None:
            lc["output_max_index"] = bool(pt.output_max_index)
    else:
        lc["type"] = "average"
        lc["average_strategy"] = {"Sum": "sum", "SumPooling": "sum", "SquareRootN": "squarerootn",
                                  "SquareRootNPooling": "squarerootn"}.get(kind, "average")
    lc["trans_type"] = _level(kw.get("agg_level"))
    lc["seq_pool_stride"] = int(kw.get("stride", -1))


def _x_batch_norm(lc, a, kw, ins, rec, name):
    """BatchNormLayer: the input three times (scale w0, moving mean w1, moving
    variance w2, the last two static), a [1, C] bias, default act relu; image_conf of
    the input (parse_image / parse_image3d), height / width (/ depth) only when the
    input has an image size."""
    src = _in_lc(rec, ins)
    three_d = bool(kw.get("img3D"))
    c = int(kw.get("num_channels") or src.get("_num_filters") or 0)
    if not c:
        xs = list(getattr(ins[0][0], "shape", []) or [])
        if len(xs) >= 4 and not src.get("height"):
            c = int(xs[1])
    if not c:
        hw = int(src.get("height", 0) or 0) * int(src.get("width", 0) or 0) * int(src.get("depth", 1) or 1)
        c = (lc["size"] // hw) if hw else lc["size"]
    lc["active_type"] = _act_or(kw, "act", "relu")
    x = ins[0][0]
    lc["inputs"] = [{"input_layer_name": rec.layer_name(x) or x.name, "input_parameter_name": f"_{name}.w{i}"}
                    for i in range(3)]
    lc["inputs"][0]["image_conf"] = _image_conf(rec, ins, c, three_d)
    lc["bias_parameter_name"] = f"_{name}.wbias"
    lc["moving_average_fraction"] = float(kw.get("moving_average_fraction", 0.9))
    lc["epsilon"] = float(kw.get("epsilon", 1e-5))
    if src.get("width") or src.get("height"):
        ic = lc["inputs"][0]["image_conf"]
        lc["height"], lc["width"], lc["depth"] = ic["img_size_y"], ic["img_size"], ic.get("img_size_z", 1)
    else:
        for k in ("height", "width", "depth"):
            lc.pop(k, None)
    lc["_num_filters"] = c
    _set_params(rec, name, lc, [(f"_{name}.w0", [c], 0.0, False), (f"_{name}.w1", [1, c], 0.0, False),
                                (f"_{name}.w2", [1, c], 0.0, False), (f"_{name}.wbias", [1, c], 0.0, False)])
    for p in rec.params:
        if p["name"] == f"_{name}.w0":
            p["initial_mean"], p["dims"] = 1.0, []  # the reference leaves the scale's dims unset
        elif p["name"] in (f"_{name}.w1", f"_{name}.w2"):
            p["is_static"] = p["is_shared"] = True


def _x_nce(lc, a, kw, ins, rec, name):
    """NCELayer: sigmoid, a [num_classes, in_size] weight on the input only (label and
    sample-weight layers carry none), a [1, num_classes] bias."""
    x, lab = ins[0][0], ins[1][0] if len(ins) > 1 else None
    nc = int(kw.get("num_classes") or (_vsize(lab) if lab is not None else 0) or 0)
    lc["active_type"] = _act_or(kw, "act", "sigmoid")
    for li in lc.get("inputs", [])[1:]:
        li.pop("input_parameter_name", None)
    lc["inputs"][0]["input_parameter_name"] = f"_{name}.w0"
    lc["bias_parameter_name"] = f"_{name}.wbias"
    lc["num_classes"] = nc
    lc["num_neg_samples"] = int(kw.get("num_neg_samples", 10))
    _set_params(rec, name, lc, [(f"_{name}.w0", [nc, _vsize(x) or 0], 1.0 / max(nc, 1) ** 0.5, True),
                                (f"_{name}.wbias", [1, nc], 0.0, False)])


def _x_conv(lc, a, kw, ins, rec, name):
    """ConvLayer (exconv / exconvt / conv3d / deconv3d): conv_conf of the input
    (parse_conv / parse_conv3d), the output image as the layer's height / width
    (/ depth), filter parameter without dims, [num_filters, 1] shared biases."""
    three_d = lc["type"] == "conv3d"
    trans = bool(kw.get("trans"))
    nf = int(kw.get("num_filters") or 0)
    g = int(kw.get("groups") or 1)
    c = _channels(kw, rec, ins)
    fs, fsy = _xy(kw, "filter_size", 1)
    for p in rec.params:
        if p["name"] == f"_{name}.w0":
            p["dims"] = []
            if p.get("initial_smart"):  # layers.py: smart init -> std sqrt(2 / (filter_size^2 C))
                p["initial_std"] = (2.0 / (fs * fs * c)) ** 0.5
                p["initial_smart"] = False
        elif p["name"] == f"_{name}.wbias":
            p["dims"] = [p["size"], 1]
    lc["num_filters"] = nf
    lc["shared_biases"] = True
    lc["_num_filters"] = nf
    st, sty = _xy(kw, "stride", 1)
    pd, pdy = _xy(kw, "padding", 0)
    cc = {"filter_size": fs, "channels": c, "stride": st, "padding": pd, "groups": g,
          "filter_channels": (nf if trans else c) // g, "caffe_mode": True, "filter_size_y": fsy,
          "padding_y": pdy, "stride_y": sty}
    if three_d:
        fsz, stz, pdz = _z(kw, "filter_size", fs), _z(kw, "stride", st), _z(kw, "padding", pd)
        w, h, d = _img_whd(rec, ins)
        cc.update(filter_size_z=fsz, padding_z=pdz, stride_z=stz)
        if trans:
            cc.update(output_x=w, output_y=h, output_z=d, img_size=_img_size(fs, w, pd, st, True),
                      img_size_y=_img_size(fsy, h, pdy, sty, True), img_size_z=_img_size(fsz, d, pdz, stz, True))
            lc["height"], lc["width"], lc["depth"] = cc["img_size_y"], cc["img_size"], cc["img_size_z"]
        else:
            cc.update(img_size=w, img_size_y=h, img_size_z=d, output_x=_out_size(w, fs, pd, st, True),
                      output_y=_out_size(h, fsy, pdy, sty, True), output_z=_out_size(d, fsz, pdz, stz, True))
            lc["height"], lc["width"], lc["depth"] = cc["output_y"], cc["output_x"], cc["output_z"]
    else:
        dl, dly = _xy(kw, "dilation", 1)
        cc.update(dilation=dl, dilation_y=dly)
        w, h = _img_wh(rec, ins, c)
        if trans:
            cc.update(output_x=w, output_y=h, img_size=_img_size(fs, w, pd, st, True, dl),
                      img_size_y=_img_size(fsy, h, pdy, sty, True, dly))
            lc["height"], lc["width"] = cc["img_size_y"], cc["img_size"]
        else:
            cc.update(img_size=w, img_size_y=h, output_x=_out_size(w, fs, pd, st, True, dl),
                      output_y=_out_size(h, fsy, pdy, sty, True, dly))
            lc["height"], lc["width"] = cc["output_y"], cc["output_x"]
    if lc.get("inputs"):
        lc["inputs"][0]["conv_conf"] = cc
    if trans:
        lc["type"] = "deconv3d" if three_d else "exconvt"
        if three_d:  # the reference sizes the deconv3d filter with num_filters / groups
            fsz = cc["filter_size_z"]
            for p in rec.params:
                if p["name"] == f"_{name}.w0":
                    p["size"] = nf * (nf // g) * fs * fsy * fsz


def _x_img_pool(lc, a, kw, ins, rec, name):
    """PoolLayer / Pool3DLayer: pool_conf (parse_pool / parse_pool3d; ceil_mode ->
    output sizes rounded up), the output image as height / width (/ depth)."""
    three_d = lc["type"] == "pool3d"
    c = _channels(kw, rec, ins)
    kw = dict(kw)
    kw.setdefault("pool_size", a[1] if len(a) > 1 else 1)
    kx, ky = _xy(kw, "pool_size", 1)
    st, sty = _xy(kw, "stride", 1)
    pd, pdy = _xy(kw, "padding", 0)
    caffe = not kw.get("ceil_mode", True)
    pc = {"pool_type": _pool_type(kw.get("pool_type")), "channels": c, "size_x": kx, "stride": st,
          "padding": pd, "size_y": ky, "stride_y": sty, "padding_y": pdy}
    if three_d:
        kz, stz, pdz = _z(kw, "pool_size", kx), _z(kw, "stride", st), _z(kw, "padding", pd)
        w, h, d = _img_whd(rec, ins)
        pc.update(size_z=kz, stride_z=stz, padding_z=pdz, img_size=w, img_size_y=h, img_size_z=d,
                  output_x=_out_size(w, kx, pd, st, caffe), output_y=_out_size(h, ky, pdy, sty, caffe),
                  output_z=_out_size(d, kz, pdz, stz, caffe))
        lc["height"], lc["width"], lc["depth"] = pc["output_y"], pc["output_x"], pc["output_z"]
    else:
        w, h = _img_wh(rec, ins, c)
        pc.update(img_size=w, img_size_y=h, output_x=_out_size(w, kx, pd, st, caffe),
                  output_y=_out_size(h, ky, pdy, sty, caffe))
        if kw.get("exclude_mode") is not None:
            pc["exclude_mode"] = bool(kw["exclude_mode"])
        lc["height"], lc["width"] = pc["output_y"], pc["output_x"]
    lc["_num_filters"] = c
    if lc.get("inputs"):
        lc["inputs"][0]["pool_conf"] = pc


def _x_cmrnorm(lc, a, kw, ins, rec, name):
    """NormLayer (cmrnorm-projection): norm_conf with scale / size, the input image."""
    c = _channels(kw, rec, ins)
    size = int(kw.get("size", a[1] if len(a) > 1 else 5))
    w, h = _img_wh(rec, ins, c)
    nc = {"norm_type": "cmrnorm-projection", "channels": c, "size": size,
          "scale": float(kw.get("scale", 0.0128)) / size, "pow": float(kw.get("power", 0.75)), "output_x": w,
          "img_size": w, "blocked": False, "output_y": h, "img_size_y": h}
    if lc.get("inputs"):
        lc["inputs"][0]["norm_conf"] = nc
    lc["height"], lc["width"] = h, w
    lc["_num_filters"] = c


def _chain(*fs):
    def f(lc, a, kw, ins, rec, name):
        for g in fs:
            g(lc, a, kw, ins, rec, name)
    return f


def _conf0(key, make):
    """Put make(...) as inputs[0][key] (a per-input sub-config of the layer)."""
    def f(lc, a, kw, ins, rec, name):
        if lc.get("inputs"):
            lc["inputs"][0][key] = make(lc, a, kw, ins, rec, name)
    return f


def _x_clip(lc, a, kw, ins, rec, name):
    lc["inputs"][0]["clip_conf"] = {"min": float(_arg(a, kw, "min", 1)), "max": float(_arg(a, kw, "max", 2))}


def _x_row_conv(lc, a, kw, ins, rec, name):
    lc["inputs"][0]["row_conv_conf"] = {"context_length": int(_arg(a, kw, "context_len", 1))}


def _x_maxout(lc, a, kw, ins, rec, name):
    c = _channels(kw, rec, ins)
    g = int(_arg(a, kw, "groups", 1))
    ic = _image_conf(rec, ins, c)
    lc["inputs"][0]["maxout_conf"] = {"image_conf": ic, "groups": g}
    lc["height"], lc["width"] = ic["img_size_y"], ic["img_size"]
    lc["_num_filters"] = c // g


def _x_pad(lc, a, kw, ins, rec, name):
    c = _channels(kw, rec, ins)
    pc, ph, pw = (list(kw.get(k) or [0, 0]) for k in ("pad_c", "pad_h", "pad_w"))
    ic = _image_conf(rec, ins, c)
    lc["inputs"][0]["pad_conf"] = {"image_conf": ic, "pad_c": pc, "pad_h": ph, "pad_w": pw}
    lc["height"], lc["width"] = ic["img_size_y"] + sum(ph), ic["img_size"] + sum(pw)
    lc["_num_filters"] = c + sum(pc)


def _x_spp(lc, a, kw, ins, rec, name):
    c = _channels(kw, rec, ins)
    ph = int(kw.get("pyramid_height") or 1)
    lc["inputs"][0]["spp_conf"] = {"image_conf": _image_conf(rec, ins, c),
                                   "pool_type": _pool_type(kw.get("pool_type")), "pyramid_height": ph}
    lc["height"], lc["width"] = 1, (4 ** ph - 1) // 3
    lc["_num_filters"] = c


def _x_roi_pool(lc, a, kw, ins, rec, name):
    pw, ph = int(kw.get("pooled_width", 1)), int(kw.get("pooled_height", 1))
    lc["inputs"][0]["roi_pool_conf"] = {"pooled_width": pw, "pooled_height": ph,
                                        "spatial_scale": float(kw.get("spatial_scale", 1.0))}
    lc["height"], lc["width"] = ph, pw
    lc["_num_filters"] = _channels(kw, rec, ins)


def _x_scale_sub_region(lc, a, kw, ins, rec, name):
    c = _channels(kw, rec, ins)
    ic = _image_conf(rec, ins, c)
    lc["inputs"][0]["scale_sub_region_conf"] = {"image_conf": ic, "value": float(_arg(a, kw, "value", 2))}
    lc["height"], lc["width"] = ic["img_size_y"], ic["img_size"]
    lc["_num_filters"] = c


def _x_bilinear(lc, a, kw, ins, rec, name):
    c = _channels(kw, rec, ins)
    ox, oy = int(kw.get("out_size_x") or 0), int(kw.get("out_size_y") or 0)
    lc["inputs"][0]["bilinear_interp_conf"] = {"image_conf": _image_conf(rec, ins, c), "out_size_x": ox,
                                               "out_size_y": oy}
    lc["height"], lc["width"] = oy, ox
    lc["_num_filters"] = c


def _x_detection_output(lc, a, kw, ins, rec, name):
    lc["inputs"][0]["detection_output_conf"] = {
        "num_classes": int(kw.get("num_classes")), "nms_threshold": float(kw.get("nms_threshold", 0.45)),
        "nms_top_k": int(kw.get("nms_top_k", 400)), "background_id": int(kw.get("background_id", 0)),
        "input_num": len(kw["input_loc"]) if isinstance(kw.get("input_loc"), (list, tuple)) else 1,
        "keep_top_k": int(kw.get("keep_top_k", 200)),
        "confidence_threshold": float(kw.get("confidence_threshold", 0.01))}


def _x_multibox_loss(lc, a, kw, ins, rec, name):
    lc["inputs"][0]["multibox_loss_conf"] = {
        "num_classes": int(kw.get("num_classes")), "overlap_threshold": float(kw.get("overlap_threshold", 0.5)),
        "neg_pos_ratio": float(kw.get("neg_pos_ratio", 3.0)), "neg_overlap": float(kw.get("neg_overlap", 0.5)),
        "background_id": int(kw.get("background_id", 0)),
        "input_num": len(kw["input_loc"]) if isinstance(kw.get("input_loc"), (list, tuple)) else 1}


def _x_prelu(lc, a, kw, ins, rec, name):
    src = _in_lc(rec, ins)
    size = int(src.get("size") or _vsize(ins[0][0]) or 0)
    ps = int(kw.get("partial_sum", 1))
    cs = kw.get("channel_shared")
    if cs is not None:
        c = _channels(kw, rec, ins)
        hw = int(src.get("height") or 0) * int(src.get("width") or 0)
        ps = hw * c if cs else hw
    lc["partial_sum"] = ps
    lc["height"], lc["width"], lc["depth"] = (int(src.get("height") or 0), int(src.get("width") or 0),
                                              int(src.get("depth") or 1))
    for p in rec.params:
        if p["name"] == f"_{name}.w0":
            p["size"], p["dims"] = size // ps, [1, size // ps]
            if p.get("initial_smart"):  # layers.py prelu_layer: ParamAttr(initial_mean=0.25, initial_std=0.0)
                p.update(initial_mean=0.25, initial_std=0.0, initial_smart=False)


def _x_reversed(lc, a, kw, ins, rec, name):
    lc["reversed"] = bool(kw.get("reverse", False))


def _conv_conf_of(cv, img_side):
    """ConvConfig of a conv / convt projection or operator over a square image."""
    fs, st, pd, c, g = cv["filter_size"], cv["stride"], cv["padding"], cv["channels"], cv.get("groups", 1)
    fy, sy = cv.get("filter_size_y") or fs, cv.get("stride_y") or st
    py = cv.get("padding_y") if cv.get("padding_y") is not None else pd
    conf = {"filter_size": fs, "channels": c, "stride": st, "padding": pd, "groups": g, "caffe_mode": True,
            "filter_size_y": fy, "padding_y": py, "stride_y": sy}
    if cv.get("trans"):
        out = (img_side - 1) * st + fs - 2 * pd
        conf.update(filter_channels=cv["num_filters"] // g, output_x=img_side, img_size=out, output_y=img_side,
                    img_size_y=(img_side - 1) * sy + fy - 2 * py)
    else:
        conf.update(filter_channels=c // g, output_x=_out_size(img_side, fs, pd, st, True), img_size=img_side,
                    output_y=_out_size(img_side, fy, py, sy, True), img_size_y=img_side)
    return conf


def _conv_out_size(cv, conf):
    return cv["num_filters"] * (conf["img_size"] * conf["img_size_y"] if cv.get("trans") else
                                conf["output_x"] * conf["output_y"])


def _x_mixed(lc, a, kw, ins, rec, name):
    """MixedLayer terms beyond plain projections: operators (operator_confs naming the
    positions of their operand inputs, which carry no parameter), context projections
    (window / trainable padding rows) and conv / convt projections (ConvConfig, a
    dimensionless filter parameter)."""
    base = name.split("@")[0]
    for i, (x, pr) in enumerate(ins):
        li = lc["inputs"][i] if i < len(lc.get("inputs", [])) else None
        if li is None or pr is None or getattr(pr, "v1_operands", None):
            continue
        if getattr(pr, "v1_context", None) is not None:
            start, length = pr.v1_context
            li["proj_conf"].update(context_start=start, context_length=length, trainable_padding=True)
            pad = max(0, -start) + max(0, start + length - 1)
            pn = li.get("input_parameter_name") or f"_{name}.w{i}"
            li["input_parameter_name"] = pn
            rec.params[:] = [p for p in rec.params if p["name"] != pn]
            rec.params.append({"name": pn, "size": pad * _vsize(x), "initial_mean": 0.0, "initial_std": 0.0,
                               "dims": [pad, _vsize(x)], "initial_strategy": 0, "initial_smart": False})
        cv = getattr(pr, "v1_conv", None)
        if cv is not None:
            side = int(round((_vsize(x) // cv["channels"]) ** 0.5))
            conf = _conv_conf_of(cv, side)
            osz = _conv_out_size(cv, conf)
            li["proj_conf"].update(type="convt" if cv.get("trans") else "conv", name=f"_{base}.w{i}",
                                   output_size=osz, conv_conf=conf, num_filters=cv["num_filters"])
            pn = li.get("input_parameter_name") or f"_{name}.w{i}"
            li["input_parameter_name"] = pn
            fs = cv["filter_size"]
            n = cv["num_filters"] * (cv["channels"] // cv.get("groups", 1)) * fs * fs
            rec.params[:] = [p for p in rec.params if p["name"] != pn]
            rec.params.append({"name": pn, "size": n, "initial_mean": 0.0,
                               "initial_std": (2.0 / (fs * fs * cv["channels"])) ** 0.5, "initial_strategy": 0,
                               "initial_smart": False})
    ops, seen = [], {}
    for i, (x, pr) in enumerate(ins):
        if pr is None or not getattr(pr, "v1_operands", None):
            continue
        if id(pr) not in seen:
            seen[id(pr)] = len(ops)
            kind, scale = getattr(pr, "v1_operator", ("dot_mul", 1.0))
            oc = {"type": kind, "input_indices": [], "input_sizes": [], "output_size": lc.get("size")}
            cv = getattr(pr, "v1_conv", None)
            if cv is not None:
                conf = _conv_conf_of(cv, int(round((_vsize(x) // cv["channels"]) ** 0.5)))
                oc.update(output_size=_conv_out_size(cv, conf), conv_conf=conf, num_filters=cv["num_filters"])
            else:
                oc["dotmul_scale"] = scale
            ops.append(oc)
        op = ops[seen[id(pr)]]
        op["input_indices"].append(i)
        op["input_sizes"].append(_vsize(x))
        if i < len(lc.get("inputs", [])):
            lc["inputs"][i].pop("input_parameter_name", None)
    if ops:
        lc["operator_confs"] = ops


def _x_block_expand(lc, a, kw, ins, rec, name):
    c = _channels(kw, rec, ins)
    bx, by = int(kw.get("block_x", 0)), int(kw.get("block_y", 0))
    sx, sy = int(kw.get("stride_x", 0)), int(kw.get("stride_y", 0))
    px, py = int(kw.get("padding_x", 0)), int(kw.get("padding_y", 0))
    ix, iy = int(kw.get("img_size_x", 0) or 0), int(kw.get("img_size_y", 0) or 0)
    lc["inputs"][0]["block_expand_conf"] = {
        "channels": c, "stride_x": sx, "stride_y": sy, "padding_x": px, "padding_y": py, "block_x": bx, "block_y": by,
        "output_x": _out_size(ix, bx, px, sx, False) if ix else 0,
        "output_y": _out_size(iy, by, py, sy, False) if iy else 0, "img_size_x": ix, "img_size_y": iy}
    lc["size"] = bx * by * c


def _x_cost_coeff(lc, a, kw, ins, rec, name):
    lc["coeff"] = float(kw.get("coeff", 1.0))


def _x_classification_cost(lc, a, kw, ins, rec, name):
    """classification_cost: coeff, and its default classification_error_evaluator over
    (prediction, label[, weight])."""
    lc["coeff"] = float(kw.get("coeff", 1.0))
    if kw.get("evaluator", True) is None or kw.get("evaluator") is False:
        return
    n = "classification_error_evaluator"
    k = sum(1 for e in rec.evaluators if e["type"] == "classification_error")
    rec.evaluators.append({"name": n if k == 0 else f"{n}_{k}", "type": "classification_error",
                           "input_layers": [x["input_layer_name"] for x in lc.get("inputs", [])]})


def _x_huber_reg(lc, a, kw, ins, rec, name):
    lc["coeff"] = float(kw.get("coeff", 1.0))
    lc["delta"] = float(kw.get("delta", 1.0))


def _x_selfnorm(lc, a, kw, ins, rec, name):
    lc["softmax_selfnorm_alpha"] = float(kw.get("softmax_selfnorm_alpha", 0.1))
    lc["coeff"] = float(kw.get("coeff", 1.0))


def _x_lambda(lc, a, kw, ins, rec, name):
    lc["NDCG_num"] = int(kw.get("NDCG_num", 5))
    lc["max_sort_size"] = int(kw.get("max_sort_size", -1))


def _x_lstm_step(lc, a, kw, ins, rec, name):
    """LstmStepLayer: gate / state activations, no input weights, a [1, 3 size]
    peephole bias (config_parser.py LstmStepLayer)."""
    lc["active_type"] = _ACT.get(_act_or(kw, "act", "tanh"), _act_or(kw, "act", "tanh"))
    lc["active_gate_type"] = _act_or(kw, "gate_act", "sigmoid")
    lc["active_state_type"] = _act_or(kw, "state_act", "tanh")
    for li in lc.get("inputs", []):
        li.pop("input_parameter_name", None)
    battr = kw.get("bias_attr")
    if battr is False:
        return
    n = 3 * int(lc["size"])
    bname = _attr_name(battr, 0) or f"_{name}.wbias"
    lc["bias_parameter_name"] = bname
    if bname not in rec.param_map:
        rec.param_map[bname] = bname
        rec.params.append({"name": bname, "size": n, "initial_mean": 0.0, "initial_std": 0.0, "dims": [1, n],
                           "initial_strategy": 0, "initial_smart": False})
        _apply_pattr(rec.params[-1], battr)


def _x_gru_step(lc, a, kw, ins, rec, name):
    """GruStepLayer: the [size, 3 size] weight belongs to the input (0) only."""
    lc["active_type"] = _ACT.get(_act_or(kw, "act", "tanh"), _act_or(kw, "act", "tanh"))
    lc["active_gate_type"] = _act_or(kw, "gate_act", "sigmoid")
    for li in lc.get("inputs", [])[1:]:
        pn = li.pop("input_parameter_name", None)
        if pn is not None and pn.startswith(f"_{name}."):
            rec.params[:] = [p for p in rec.params if p["name"] != pn]
            rec.param_map.pop(pn, None)


def _x_get_output(lc, a, kw, ins, rec, name):
    """GetOutputLayer: the input names which output of the source layer it reads."""
    arg = _arg(a, kw, "arg_name", 1)
    if lc.get("inputs") and arg:
        lc["inputs"][0]["input_layer_argument"] = arg


def _x_embedding(lc, a, kw, ins, rec, name):
    """embedding_layer: a mixed layer over one table projection."""
    if lc.get("inputs"):
        lc["inputs"][0]["proj_conf"] = {"type": "table", "name": f"_{name.split('@')[0]}.w0",
                                        "input_size": _vsize(ins[0][0]), "output_size": lc["size"]}


_EXTRA = {
    "embedding_layer": _x_embedding,
    "lstm_step_layer": _x_lstm_step, "gru_step_layer": _x_gru_step, "gru_step_naive_layer": _x_gru_step,
    "get_output_layer": _x_get_output,
    "batch_norm_layer": _x_batch_norm, "nce_layer": _x_nce, "img_conv_layer": _x_conv,
    "pooling_layer": _x_pooling, "slope_intercept_layer": _x_slope, "scaling_layer": _x_weight_first,
    "interpolation_layer": _x_weight_first, "power_layer": _x_weight_first,
    "ctc_layer": _x_ctc, "warp_ctc_layer": _x_ctc, "cos_sim": _x_cos, "tensor_layer": _x_tensor,
    "cross_entropy_with_selfnorm": _chain(_x_no_size, _x_selfnorm), "cross_entropy_over_beam": _x_beam,
    "detection_output_layer": _chain(_x_reorder(("priorbox", "input_loc", "input_conf"),
                                                lambda kw: int(kw.get("keep_top_k", 200)) * 7),
                                     _x_detection_output),
    "multibox_loss_layer": _chain(_x_reorder(("priorbox", "label", "input_loc", "input_conf")), _x_multibox_loss),
    "clip_layer": _x_clip, "row_conv_layer": _x_row_conv, "maxout_layer": _x_maxout, "pad_layer": _x_pad,
    "spp_layer": _x_spp, "roi_pool_layer": _x_roi_pool, "scale_sub_region_layer": _x_scale_sub_region,
    "bilinear_interp_layer": _x_bilinear, "prelu_layer": _x_prelu, "recurrent_layer": _x_reversed,
    "crf_layer": _x_cost_coeff, "rank_cost": _x_cost_coeff, "cross_entropy": _x_cost_coeff,
    "huber_regression_cost": _x_huber_reg, "huber_classification_cost": _x_cost_coeff,
    "multi_binary_label_cross_entropy": _x_cost_coeff, "sum_cost": _x_cost_coeff,
    "classification_cost": _x_classification_cost, "square_error_cost": _x_cost_coeff, "regression_cost": _x_cost_coeff,
    "mse_cost": _x_cost_coeff, "lambda_cost": _x_lambda, "mixed_layer": _x_mixed,
    "block_expand_layer": _x_block_expand,
    "img_conv3d_layer": _x_conv, "img_pool_layer": _x_img_pool, "img_pool3d_layer": _x_img_pool,
    "img_cmrnorm_layer": _x_cmrnorm,
    "factorization_machine": _x_factor, "smooth_l1_cost": _x_coeff, "kmax_seq_score_layer": _x_kmax,
    "sampling_id_layer": _x_same_size, "scale_shift_layer": _x_scale_shift, "seq_slice_layer": _x_seq_slice,
    "data_layer": _x_data, "addto_layer": _x_addto, "concat_layer": _x_concat,
    "last_seq": _x_seqins(False), "first_seq": _x_seqins(True), "expand_layer": _x_expand,
    "repeat_layer": _x_repeat, "lstmemory": _x_lstm, "grumemory": _x_gru, "hsigmoid": _x_hsigmoid,
    "selective_fc_layer": _x_selective_fc,
}


def _prod(xs):
    r = 1
    for x in xs:
        r *= int(x)
    return r


def _dfs_inputs(rec, out_names):
    """networks.outputs: data layers in DFS post-order from each output over parents."""
    seen, order = set(), []

    def visit(n):
        if n in seen:
            return
        seen.add(n)
        for p in rec.parents.get(n, []):
            visit(p)
        if rec.by_name.get(n, {}).get("type") == "data":
            order.append(n)

    for o in out_names:
        visit(o)
    return order


def model_config(rec, outputs, first_outputs=None):
    out_names = [rec.layer_name(o) or getattr(o, "name", str(o)) for o in outputs]
    names = [lc["name"] for lc in rec.layers]
    # input layers: DFS from the outputs of the first outputs(...) call (the reference
    # sets input_layer_names once, there)
    src = [rec.layer_name(o) or getattr(o, "name", str(o)) for o in (first_outputs or outputs)]
    ins = _dfs_inputs(rec, src) if src and all(o in rec.by_name for o in src) else rec.inputs
    root = [n for n in names if n not in rec.inner]
    mc = {"type": "recurrent_nn" if rec.sub_models else "nn", "layers": rec.layers, "parameters": rec.params,
          "input_layer_names": ins, "output_layer_names": out_names, "evaluators": rec.evaluators,
          "sub_models": [{"name": "root", "layer_names": root, "input_layer_names": ins,
                          "output_layer_names": out_names, "evaluator_names": [e["name"] for e in rec.evaluators],
                          "is_recurrent_layer_group": False}] + list(rec.sub_models)}
    return _proto2_clean(mc)


def _proto2_clean(d):
    """proto2: an empty repeated field is an absent one; "_"-prefixed keys are the
    recorder's own bookkeeping, not message fields."""
    if isinstance(d, dict):
        return {k: _proto2_clean(v) for k, v in d.items()
                if not k.startswith("_") and not (isinstance(v, list) and not v)}
    if isinstance(d, list):
        return [_proto2_clean(x) for x in d]
    return d


_METHOD = {"Momentum": "momentum", "Adam": "adam", "Adamax": "adamax", "AdaGrad": "adagrad",
           "DecayedAdaGrad": "decayed_adagrad", "AdaDelta": "adadelta", "RMSProp": "rmsprop"}


def opt_config(cfg):
    """OptimizationConfig as the reference's settings() leaves it: every field it
    assigns, at its default unless the config set it (optimizers.py settings /
    config_parser.py default_optimization_config)."""
    m = cfg.get("learning_method")
    kind = getattr(getattr(m, "kind", None), "__name__", "Momentum")
    ex = cfg.get("extra") or {}
    oc = {"batch_size": int(cfg.get("batch_size") or 1), "algorithm": "sgd",
          "learning_rate": float(cfg.get("learning_rate") or 1e-3),
          "learning_rate_decay_a": float(ex.get("learning_rate_decay_a", 0.0)),
          "learning_rate_decay_b": float(ex.get("learning_rate_decay_b", 0.0)), "l1weight": 0.1, "l2weight": 0.0,
          "c1": 0.0001, "backoff": 0.5, "owlqn_steps": 10, "max_backoff": 5, "l2weight_zero_iter": 0,
          "average_window": 0.0, "learning_method": _METHOD.get(kind, "momentum"), "ada_epsilon": 1e-6,
          "do_average_in_cpu": False, "ada_rou": 0.95,
          "learning_rate_schedule": str(ex.get("learning_rate_schedule", "poly")), "delta_add_rate": 1.0,
          "shrink_parameter_value": 0.0, "adam_beta1": 0.9, "adam_beta2": 0.999, "adam_epsilon": 1e-8,
          "learning_rate_args": str(ex.get("learning_rate_args", "")), "async_lagged_grad_discard_ratio": 1.5}
    kw = getattr(m, "kw", {}) or {}
    if kind == "Adam":
        oc.update(adam_beta1=kw.get("beta1", 0.9), adam_beta2=kw.get("beta2", 0.999),
                  adam_epsilon=kw.get("epsilon", 1e-8))
    elif kind in ("AdaGrad", "DecayedAdaGrad", "AdaDelta", "RMSProp"):
        if kw.get("epsilon") is not None:
            oc["ada_epsilon"] = float(kw["epsilon"])
        if kw.get("rho") is not None:
            oc["ada_rou"] = float(kw["rho"])
    reg = cfg.get("regularization")
    rate = getattr(reg, "rate", None) or getattr(reg, "regularization_coeff", None)
    if rate:
        oc["l2weight"] = float(rate)
    if cfg.get("gradient_clipping_threshold"):
        oc["gradient_clipping_threshold"] = float(cfg["gradient_clipping_threshold"])
    return oc


def data_configs(cfg):
    src = cfg.get("data_sources")
    if not src:
        return None, None
    train, test, module, obj, args = (src["train_list"], src["test_list"], src["module"], src["obj"],
                                      src.get("args"))

    def pick(v, i):  # define_py_data_sources2: a (train, test) pair of modules / objects / args
        return v[i] if isinstance(v, (list, tuple)) else v

    def dc(files, for_test):
        if not files:
            return None
        i = int(for_test)
        a = pick(args, i)
        return {"type": "py2", "files": files, "async_load_data": False, "for_test": for_test,
                "load_data_module": pick(module, i), "load_data_object": pick(obj, i),
                "load_data_args": "" if a is None else str(a), "data_ratio": 1, "is_main_data": True,
                "usage_ratio": 1.0}

    return dc(train, False), dc(test, True)
