"""Every reference v1 config (python/paddle/trainer_config_helpers/tests/configs/*.py,
run UNMODIFIED through ``parse_config`` as the reference's own test harness does) against
its expected ModelConfig (protostr/*.protostr, text format read as data) -- the full
message, field by field, with proto2 semantics (an empty repeated field is absent;
floats compared to 1e-6 relative).  VERDICT r4 item 9.

The comparison is STRICT: every field of the reference text must be in the recorder's
schema (a field the schema does not know is kept as "?<name>" and reported), so a
match covers the whole message -- conv / pool / norm / image sub-configs, evaluators,
and for the TrainerConfig-rooted fixtures (test_split_datasource) the optimisation /
data sections.  The test pins the configs that already match exactly and the number
that parse, so the v1 layer recorder (trainer_config_helpers/config_proto.py) can only
improve.  Recurrent groups are recorded as the reference's sub-models (scatter /
gather / memory agents, in / out links); all 56 reference configs that parse match."""
import glob
import os

import pytest

REF = "/root/reference/python/paddle/trainer_config_helpers/tests/configs"

pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference configs not mounted")

# configs whose whole ModelConfig matches the reference's protostr today
EXACT = {
    "img_layers", "img_trans_layers", "last_first_seq", "layer_activations", "math_ops", "shared_fc",
    "simple_rnn_layers", "test_BatchNorm3D", "test_bi_grumemory", "test_bilinear_interp", "test_clip_layer",
    "test_conv3d_layer", "test_cost_layers", "test_cost_layers_with_weight", "test_cross_entropy_over_beam",
    "test_deconv3d_layer", "test_detection_output_layer", "test_dot_prod_layer", "test_expand_layer",
    "test_factorization_machine", "test_fc", "test_gated_unit_layer", "test_grumemory_layer", "test_hsigmoid",
    "test_kmax_seq_socre_layer", "test_l2_distance_layer", "test_lstmemory_layer", "test_maxout",
    "test_multibox_loss_layer", "test_multiplex_layer", "test_ntm_layers", "test_pad", "test_pooling3D_layer",
    "test_prelu_layer", "test_print_layer", "test_recursive_topology", "test_repeat_layer", "test_resize_layer",
    "test_roi_pool_layer", "test_row_conv", "test_row_l2_norm_layer", "test_scale_shift_layer",
    "test_scale_sub_region_layer", "test_seq_concat_reshape", "test_seq_slice_layer", "test_sequence_pooling",
    "test_smooth_l1", "test_split_datasource", "test_spp_layer", "test_sub_nested_seq_select_layer", "unused_layers",
    "util_layers", "test_rnn_group", "shared_gru", "shared_lstm", "projections",
}
# all but test_config_parser_for_non_file_config (a stdin driver script, not a
# config) and test_crop (outputs an undefined layer)
MIN_PARSED = 56


def _diff(a, b, path=""):
    out = []
    if isinstance(a, dict) and isinstance(b, dict):
        for k in sorted(set(a) | set(b)):
            if k not in a:
                out.append(f"{path}/{k} missing")
            elif k not in b:
                out.append(f"{path}/{k} extra")
            else:
                out += _diff(a[k], b[k], f"{path}/{k}")
    elif isinstance(a, list) and isinstance(b, list):
        if len(a) != len(b):
            out.append(f"{path} len {len(a)} vs {len(b)}")
        for i, (x, y) in enumerate(zip(a, b)):
            out += _diff(x, y, f"{path}[{i}]")
    elif isinstance(a, float) or isinstance(b, float):
        try:
            if abs(float(a) - float(b)) > 1e-6 * max(1.0, abs(float(b))):
                out.append(f"{path} {a!r} vs {b!r}")
        except (TypeError, ValueError):
            out.append(f"{path} {a!r} vs {b!r}")
    elif a != b:
        out.append(f"{path} {a!r} vs {b!r}")
    return out


def _results():
    import paddle_amd.trainer_config_helpers as tch
    from paddle_amd.trainer_config_helpers import config_proto as cp

    res = {}
    for f in sorted(glob.glob(os.path.join(REF, "*.py"))):
        n = os.path.basename(f)[:-3]
        try:
            got = tch.parse_config(f).model_config()
        except Exception as e:  # noqa: BLE001 -- the census records every failure
            res[n] = ("parse-error", repr(e)[:200])
            continue
        p = os.path.join(REF, "protostr", n + ".protostr")
        if not os.path.exists(p):
            res[n] = ("no-protostr", "")
            continue
        with open(p) as fh:
            txt = fh.read()
        if txt.lstrip().startswith("model_config"):  # a whole TrainerConfig fixture
            exp = cp.from_text("TrainerConfig", txt, strict=True)
            got = tch.parse_config(f).trainer_config()
        else:
            exp = cp.from_text("ModelConfig", txt, strict=True)
        d = _diff(got, exp)
        res[n] = ("exact", "") if not d else ("diff", f"{len(d)}: {d[:3]}")
    return res


def test_reference_v1_configs_parse_and_match():
    res = _results()
    assert len(res) >= 56
    parsed = [n for n, (st, _) in res.items() if st != "parse-error"]
    exact = {n for n, (st, _) in res.items() if st == "exact"}
    assert len(parsed) >= MIN_PARSED, {n: m for n, (st, m) in res.items() if st == "parse-error"}
    lost = EXACT - exact
    assert not lost, {n: res[n] for n in lost}
