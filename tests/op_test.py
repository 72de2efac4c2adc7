"""OpTest harness (reference: python/paddle/fluid/tests/unittests/op_test.py).

* ``check_output``: builds a one-op Program, runs it with the Executor on every
  available place (CPU, plus the HIP device when present) and compares with the
  numpy expectation.
* ``check_grad``: analytic gradients from ``append_backward`` (grad op makers +
  grad kernels, or the registry's automatic VJP) vs. numeric central differences
  (delta 0.005) of ``mean(mean(out_i))``, within ``max_relative_error`` -- the
  reference's get_numeric_gradient (op_test.py:43) / check_grad (:395) contract.
"""
from __future__ import annotations

import numpy as np
import torch

import paddle_amd.fluid as fluid
from paddle_amd.framework import core
from paddle_amd.framework import registry as R


def _places():
    ps = [core.CPUPlace()]
    if torch.cuda.is_available():
        ps.append(core.CUDAPlace(0))
    return ps


def _norm_inputs(inputs):
    """slot -> list of (name, ndarray, lod)"""
    out = {}
    for slot, v in inputs.items():
        if isinstance(v, list):
            out[slot] = [(n, a[0] if isinstance(a, tuple) else a, a[1] if isinstance(a, tuple) else None)
                         for n, a in v]
        elif isinstance(v, tuple):
            out[slot] = [(slot.lower(), v[0], v[1])]
        else:
            out[slot] = [(slot.lower(), v, None)]
    return out


class OpTest:
    op_type = None
    inputs = {}
    outputs = {}
    attrs = {}

    def _build(self, place_outputs=True):
        prog, startup = fluid.Program(), fluid.Program()
        ins = _norm_inputs(self.inputs)
        feed = {}
        with fluid.program_guard(prog, startup):
            blk = prog.global_block()
            in_vars = {}
            for slot, lst in ins.items():
                vs = []
                for name, arr, lod in lst:
                    arr = np.asarray(arr)
                    v = blk.create_var(name=name, shape=list(arr.shape), dtype=arr.dtype, lod_level=len(lod or []),
                                       stop_gradient=False)
                    vs.append(v)
                    t = core.LoDTensor()
                    t.set(arr)
                    if lod:
                        t.set_recursive_sequence_lengths(lod)
                    feed[name] = t
                in_vars[slot] = vs
            out_vars = {}
            for slot, v in self.outputs.items():
                if isinstance(v, list):
                    out_vars[slot] = [blk.create_var(name=n, dtype=np.asarray(a if not isinstance(a, tuple) else a[0]).dtype)
                                      for n, a in v]
                else:
                    a = v[0] if isinstance(v, tuple) else v
                    out_vars[slot] = [blk.create_var(name=slot.lower() + "_out", dtype=np.asarray(a).dtype)]
            info = R.get_op_info(self.op_type)
            for s in info.outputs:
                if s.name not in out_vars:
                    out_vars[s.name] = [blk.create_var(name=s.name.lower() + "_extra")]
            op = blk.append_op(type=self.op_type, inputs=in_vars, outputs=out_vars, attrs=dict(self.attrs))
        return prog, startup, feed, in_vars, out_vars, op

    def check_output(self, atol=1e-5, rtol=1e-5, places=None, no_check_set=(), exec_only=False):
        for place in places or _places():
            prog, _, feed, _, out_vars, _ = self._build()
            fetch = []
            expect = []
            for slot, v in self.outputs.items():
                if slot in no_check_set:
                    continue
                if isinstance(v, list):
                    for (n, a), var in zip(v, out_vars[slot]):
                        fetch.append(var)
                        expect.append(a[0] if isinstance(a, tuple) else a)
                else:
                    fetch.append(out_vars[slot][0])
                    expect.append(v[0] if isinstance(v, tuple) else v)
            exe = fluid.Executor(place)
            got = exe.run(prog, feed=feed, fetch_list=fetch, scope=core.Scope())
            if exec_only:
                assert all(np.all(np.isfinite(np.asarray(g, dtype=np.float64))) for g in got
                           if np.asarray(g).dtype.kind == "f")
                continue
            for g, e, var in zip(got, expect, fetch):
                e = np.asarray(e)
                g = np.asarray(g).reshape(e.shape) if np.asarray(g).size == e.size else np.asarray(g)
                np.testing.assert_allclose(g.astype(np.float64) if g.dtype != bool else g,
                                           e.astype(np.float64) if e.dtype != bool else e, atol=atol, rtol=rtol,
                                           err_msg=f"{self.op_type}:{var.name} on {place}")

    def _numeric_grad(self, feed, in_name, output_slots, delta):
        info = R.get_op_info(self.op_type)
        ins = _norm_inputs(self.inputs)

        def loss(fd):
            ctx_ins = {slot: [core.LoDTensor(torch.from_numpy(np.asarray(fd[n].numpy(), dtype=np.float64))
                                             if np.asarray(fd[n].numpy()).dtype.kind == "f"
                                             else torch.from_numpy(np.asarray(fd[n].numpy())), fd[n].lod())
                              for n, _, _ in lst] for slot, lst in ins.items()}
            outs = {s.name: [f"{s.name}#{i}" for i in range(4)] for s in info.outputs}
            ctx = R.KernelContext(self.op_type, ctx_ins, outs, dict(info.attrs, **self.attrs))
            R.run_kernel(info, ctx)
            vals = []
            for slot in output_slots:
                for r in ctx.results[slot]:
                    t = r.tensor if isinstance(r, core.LoDTensor) else r
                    vals.append(t.double().mean().item())
            return float(np.mean(vals))

        base = feed[in_name].numpy().astype(np.float64)
        grad = np.zeros_like(base)
        flat = base.reshape(-1)
        for i in range(flat.size):
            orig = flat[i]
            flat[i] = orig + delta
            fd = dict(feed)
            fd[in_name] = core.LoDTensor(torch.from_numpy(flat.reshape(base.shape).copy()), feed[in_name].lod())
            yp = loss(fd)
            flat[i] = orig - delta
            fd[in_name] = core.LoDTensor(torch.from_numpy(flat.reshape(base.shape).copy()), feed[in_name].lod())
            ym = loss(fd)
            flat[i] = orig
            grad.reshape(-1)[i] = (yp - ym) / (2 * delta)
        return grad

    def check_grad(self, inputs_to_check, output_names, max_relative_error=0.005, no_grad_set=None,
                   numeric_grad_delta=0.005, places=None):
        if isinstance(output_names, str):
            output_names = [output_names]
        for place in places or _places():
            prog, startup, feed, in_vars, out_vars, op = self._build()
            name_of = {}
            for slot, vs in in_vars.items():
                for v in vs:
                    name_of[v.name] = v
            with fluid.program_guard(prog, startup):
                means = [fluid.layers.mean(v) for slot in output_names for v in out_vars[slot]]
                loss = fluid.layers.mean(fluid.layers.sums(means)) if len(means) > 1 else means[0]
                # mean(mean(out_i)) over outputs == reference loss definition
                if len(means) > 1:
                    loss = fluid.layers.scale(fluid.layers.sums(means), scale=1.0 / len(means))
                fluid.backward.append_backward(loss, no_grad_set=set(no_grad_set or []))
            # feed float64 for CPU precision
            feed64 = {}
            for k, t in feed.items():
                a = t.numpy()
                if a.dtype.kind == "f" and isinstance(place, core.CPUPlace):
                    a = a.astype(np.float64)
                nt = core.LoDTensor()
                nt.set(a)
                nt.set_lod(t.lod())
                feed64[k] = nt
            for v in prog.global_block().vars.values():
                if feed64.get(v.name) is not None and feed64[v.name].numpy().dtype == np.float64:
                    v.dtype = core.VT.FP64
            names = []
            for n in inputs_to_check:
                cand = [v for v in name_of if v == n or v == n.lower()]
                names.append(cand[0] if cand else n)
            grads = [prog.global_block()._find_var_recursive(n + "@GRAD") for n in names]
            exe = fluid.Executor(place)
            got = exe.run(prog, feed=feed64, fetch_list=grads, scope=core.Scope())
            for n, g in zip(names, got):
                num = self._numeric_grad(feed64, n, output_names, numeric_grad_delta)
                a = np.asarray(g, dtype=np.float64).reshape(num.shape)
                abs_a = np.abs(num)
                abs_a[abs_a < 1e-3] = 1
                diff = np.abs(a - num) / abs_a
                assert diff.max() <= max_relative_error, (
                    f"{self.op_type} grad {n} on {place}: max rel err {diff.max():.3g} > {max_relative_error}")
