"""Native parameter optimizer (csrc/runtime/param_optimizer.cc; reference
paddle/legacy/optimizer/*_optimizer.cc, parameter_optimizer_test.cc): each update
rule against a float64 numpy transcription, the Linear learning-rate policy, state
serialisation / resume (exact), and the reference's per-element decimal TensorProto
form on load."""
import numpy as np
import pytest

from paddle_amd.distributed import param_optimizer as PO
from paddle_amd.trainer_config_helpers import config_proto as cp


def _ref(kind, p, gs, lr, lr_at=None, **kw):
    p = p.astype(np.float64).copy()
    a0, a1, a2 = np.zeros_like(p), np.zeros_like(p), np.zeros_like(p)
    for n, g in enumerate(gs, 1):
        g = g.astype(np.float64)
        r = lr_at(n) if lr_at else lr
        dec = kw.get("decay", 0.0)
        if kind == "sgd":
            mu = kw.get("momentum", 0.0)
            if mu == 0.0:
                v = -r * g - r * dec * p
            else:
                a0 = mu * a0 - r * g - r * dec * p
                v = a0
            p = p + mu * v - r * g if kw.get("nesterov") else p + v
        elif kind == "adadelta":
            rho, eps = kw.get("rho", 0.9), kw.get("epsilon", 1e-5)
            a0 = rho * a0 + (1 - rho) * g * g
            a2 = np.sqrt(a1 + eps) / np.sqrt(a0 + eps) * g
            a1 = rho * a1 + (1 - rho) * a2 * a2
            p = p - r * a2 - r * dec * p
        elif kind == "adagrad":
            eps = kw.get("epsilon", 1e-5)
            a0 = a0 + g * g
            p = p - r * g / np.sqrt(a0 + eps) - r * dec * p
        else:
            # AdamConfig declares no proto defaults: unset fields read as 0
            b1, b2, eps = kw.get("beta_1", 0.0), kw.get("beta_2", 0.0), kw.get("epsilon", 0.0)
            a0 = b1 * a0 + (1 - b1) * g
            a1 = b2 * a1 + (1 - b2) * g * g
            p = p - r * np.sqrt(1 - b2 ** n) / (1 - b1 ** n) * (a0 / np.sqrt(a1 + eps) + dec * p)
    return p


CASES = [("sgd", {}), ("sgd", {"momentum": 0.9, "decay": 1e-3}), ("sgd", {"momentum": 0.9, "nesterov": True}),
         ("adadelta", {"rho": 0.95}), ("adagrad", {"decay": 1e-4}),
         ("adam", {"beta_1": 0.8, "beta_2": 0.99, "epsilon": 1e-8, "decay": 1e-3}), ("adam", {})]


@pytest.mark.parametrize("kind,kw", CASES)
def test_update_rules_match_numpy(kind, kw):
    rs = np.random.RandomState(0)
    p0 = rs.randn(37).astype("float32")
    gs = [rs.randn(37).astype("float32") for _ in range(5)]
    o = PO.ParameterOptimizer(PO.optimizer_config(kind, lr=0.05, **kw), p0)
    for g in gs:
        o.update(g)
    np.testing.assert_allclose(o.weights(), _ref(kind, p0, gs, 0.05, **kw), rtol=1e-5, atol=1e-6)


def test_linear_lr_policy_and_state_resume():
    rs = np.random.RandomState(1)
    p0 = rs.randn(64).astype("float32")
    gs = [rs.randn(64).astype("float32") for _ in range(6)]
    cfg = PO.optimizer_config("adam", lr=0.1, lr_policy="linear", lr_decay_a=0.01, lr_decay_b=0.05, beta_1=0.9,
                              beta_2=0.999, epsilon=1e-8)
    full = PO.ParameterOptimizer(cfg, p0)
    for g in gs:
        full.update(g)
    half = PO.ParameterOptimizer(cfg, p0)
    for g in gs[:3]:
        half.update(g)
    st = half.state()
    resumed = PO.ParameterOptimizer(cfg, np.zeros_like(p0), state=st)  # parameter comes from the state
    for g in gs[3:]:
        resumed.update(g)
    np.testing.assert_array_equal(resumed.weights(), full.weights())
    np.testing.assert_allclose(full.weights(), _ref("adam", p0, gs, 0.1, lr_at=lambda n: max(0.1 - 0.01 * n, 0.05), beta_1=0.9,
                                                    beta_2=0.999, epsilon=1e-8),
                               rtol=1e-5, atol=1e-6)


def test_reads_decimal_tensor_proto_state():
    """The reference serialises TensorProto.content as one decimal string per element."""
    p = np.array([1.5, -2.25, 3.0], np.float32)
    m = np.array([0.5, 0.25, -1.0], np.float32)
    cp._S.setdefault("TensorProto", [("data_type", 1, "int32", 0), ("content", 2, "string", 1)])
    cp._FIELDS["TensorProto"] = {f[0]: f for f in cp._S["TensorProto"]}
    cp._BYNUM["TensorProto"] = {f[1]: f for f in cp._S["TensorProto"]}
    cp._S["SGDOptimizerState"] = [("lr_state", 101, "LrPolicyState", 0), ("num_sample_passed", 104, "double", 0),
                                  ("parameter", 1, "TensorProto", 0), ("momentums", 2, "TensorProto", 0)]
    cp._S["LrPolicyState"] = [("learning_rate", 1, "double", 0)]
    for mname in ("SGDOptimizerState", "LrPolicyState"):
        cp._FIELDS[mname] = {f[0]: f for f in cp._S[mname]}
        cp._BYNUM[mname] = {f[1]: f for f in cp._S[mname]}
    st = cp.encode("SGDOptimizerState", {
        "lr_state": {"learning_rate": 0.1}, "num_sample_passed": 3.0,
        "parameter": {"data_type": 4, "content": [repr(float(x)) for x in p]},
        "momentums": {"data_type": 4, "content": [repr(float(x)) for x in m]}})
    o = PO.ParameterOptimizer(PO.optimizer_config("sgd", lr=0.1, momentum=0.5), np.zeros(3, np.float32), state=st)
    np.testing.assert_array_equal(o.weights(), p)
    g = np.ones(3, np.float32)
    o.update(g)
    np.testing.assert_allclose(o.weights(), p + (0.5 * m - 0.1 * g), rtol=1e-6)


def test_go_pserver_runs_the_native_optimizer(tmp_path):
    """distributed/pserver.py with an OptimizerConfig-carrying parameter config: the
    updates go through the native library, and the CRC-checked checkpoint resumes the
    native optimizer state exactly."""
    from paddle_amd.distributed import master, pserver as PS

    store = PS.KVStore(str(tmp_path / "kv.json"))
    svc = PS.PServerService(index=0, checkpoint_interval=0, checkpoint_dir=str(tmp_path), store=store)
    rs = np.random.RandomState(2)
    w0 = rs.randn(5, 6).astype("float32")
    cfg = {"optimizer_config": PO.optimizer_config("adam", lr=0.02, beta_1=0.85, beta_2=0.999, epsilon=1e-8).hex()}
    svc.init_param("w", PS._enc(w0), cfg)
    svc.finish_init_params()
    ref = PO.ParameterOptimizer(PO.optimizer_config("adam", lr=0.02, beta_1=0.85, beta_2=0.999, epsilon=1e-8), w0)
    gs = [rs.randn(5, 6).astype("float32") for _ in range(4)]
    for g in gs[:2]:
        svc.send_grad("w", PS._enc(g))
        ref.update(g)
    np.testing.assert_array_equal(PS._dec(svc.get_param("w")), ref.weights())
    svc.checkpoint()
    back = PS.load_checkpoint(store, 0)
    svc2 = PS.PServerService(index=0, checkpoint=back)
    for g in gs[2:]:
        svc2.send_grad("w", PS._enc(g))
        ref.update(g)
    np.testing.assert_array_equal(PS._dec(svc2.get_param("w")), ref.weights())


def test_unset_learning_rate_is_const_lr_one():
    """lr_policy unset reads as Const and ConstLrConfig.learning_rate defaults to 1.0
    (reference parameter_optimizer.cc:32-43; its ConstLr(0.1) branch is unreachable)."""
    rs = np.random.RandomState(3)
    p0 = rs.randn(9).astype("float32")
    g = rs.randn(9).astype("float32")
    o = PO.ParameterOptimizer(cp.encode("OptimizerConfig", {"optimizer": 1}), p0)
    o.update(g)
    np.testing.assert_allclose(o.weights(), p0 - g, rtol=1e-6, atol=1e-6)
