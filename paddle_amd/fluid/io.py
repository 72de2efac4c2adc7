"""Checkpoint / inference-model IO (python/paddle/fluid/io.py:89-677).

Builds a temporary program of ``save``/``load`` (one file per var) or
``save_combine``/``load_combine`` (one file) ops and runs it, exactly like the
reference, so files are byte-compatible LoDTensor streams; ``__model__`` is the
serialized pruned ProgramDesc.
"""
from __future__ import annotations

import os

from ..framework import core
from . import unique_name
from .executor import Executor, global_scope
from .framework import Parameter, Program, Variable, default_main_program, program_guard


def is_parameter(var):
    return isinstance(var, Parameter)


def is_persistable(var):
    if var.type in (core.VT.FEED_MINIBATCH, core.VT.FETCH_LIST, core.VT.READER, core.VT.RAW):
        return False
    return var.persistable


def _clone_var_in_block_(block, var):
    return block.create_var(name=var.name, shape=var.shape, dtype=var.dtype, type=var.type,
                            lod_level=var.lod_level, persistable=True)


def save_vars(executor, dirname, main_program=None, vars=None, predicate=None, filename=None):
    if vars is None:
        if main_program is None:
            main_program = default_main_program()
        vars = [v for v in main_program.list_vars() if predicate is None or predicate(v)]
        return save_vars(executor, dirname, main_program, vars, None, filename)
    save_program = Program()
    save_block = save_program.global_block()
    save_var_list = []
    for each in vars:
        if each.type == core.VT.RAW:
            continue
        nv = _clone_var_in_block_(save_block, each)
        if filename is None:
            save_block.append_op(type="save", inputs={"X": [nv]}, outputs={},
                                 attrs={"file_path": os.path.join(dirname, nv.name)})
        else:
            save_var_list.append(nv)
    if filename is not None:
        save_var_list.sort(key=lambda v: v.name)
        save_block.append_op(type="save_combine", inputs={"X": save_var_list}, outputs={},
                             attrs={"file_path": os.path.join(dirname, filename)})
    if dirname:
        os.makedirs(dirname, exist_ok=True)
    executor.run(save_program)


def save_params(executor, dirname, main_program=None, filename=None):
    save_vars(executor, dirname, main_program, vars=None, predicate=is_parameter, filename=filename)


def save_persistables(executor, dirname, main_program=None, filename=None):
    save_vars(executor, dirname, main_program, vars=None, predicate=is_persistable, filename=filename)


def load_vars(executor, dirname, main_program=None, vars=None, predicate=None, filename=None):
    if vars is None:
        if main_program is None:
            main_program = default_main_program()
        vars = [v for v in main_program.list_vars() if predicate is None or predicate(v)]
        return load_vars(executor, dirname, main_program, vars, None, filename)
    load_prog = Program()
    load_block = load_prog.global_block()
    load_var_list = []
    for each in vars:
        if each.type == core.VT.RAW:
            continue
        nv = _clone_var_in_block_(load_block, each)
        if filename is None:
            load_block.append_op(type="load", inputs={}, outputs={"Out": [nv]},
                                 attrs={"file_path": os.path.join(dirname, nv.name)})
        else:
            load_var_list.append(nv)
    if filename is not None:
        load_var_list.sort(key=lambda v: v.name)
        load_block.append_op(type="load_combine", inputs={}, outputs={"Out": load_var_list},
                             attrs={"file_path": os.path.join(dirname, filename)})
    executor.run(load_prog)


def load_params(executor, dirname, main_program=None, filename=None):
    load_vars(executor, dirname, main_program, predicate=is_parameter, filename=filename)


def load_persistables(executor, dirname, main_program=None, filename=None):
    load_vars(executor, dirname, main_program, predicate=is_persistable, filename=filename)


def get_inference_program(target_vars, main_program=None):
    if main_program is None:
        main_program = default_main_program()
    if not isinstance(target_vars, list):
        target_vars = [target_vars]
    return main_program.clone(for_test=True).prune(target_vars)


def prepend_feed_ops(inference_program, feed_target_names, feed_holder_name="feed"):
    gb = inference_program.global_block()
    feed_var = gb.create_var(name=feed_holder_name, type=core.VT.FEED_MINIBATCH, persistable=True)
    for i, name in enumerate(feed_target_names):
        out = gb.var(name)
        gb.prepend_op(type="feed", inputs={"X": [feed_var]}, outputs={"Out": [out]}, attrs={"col": i})


def append_fetch_ops(inference_program, fetch_target_names, fetch_holder_name="fetch"):
    gb = inference_program.global_block()
    fetch_var = gb.create_var(name=fetch_holder_name, type=core.VT.FETCH_LIST, persistable=True)
    for i, name in enumerate(fetch_target_names):
        gb.append_op(type="fetch", inputs={"X": [name]}, outputs={"Out": [fetch_var]}, attrs={"col": i})


def save_inference_model(dirname, feeded_var_names, target_vars, executor, main_program=None,
                         model_filename=None, params_filename=None, export_for_deployment=True):
    if isinstance(feeded_var_names, str):
        feeded_var_names = [feeded_var_names]
    if isinstance(target_vars, Variable):
        target_vars = [target_vars]
    if main_program is None:
        main_program = default_main_program()
    os.makedirs(dirname, exist_ok=True)
    inference_program = main_program.clone(for_test=True).prune(target_vars)
    gb = inference_program.global_block()
    gb.ops = [op for op in gb.ops if op.type not in ("feed", "fetch")]
    prepend_feed_ops(inference_program, feeded_var_names)
    append_fetch_ops(inference_program, [t.name for t in target_vars])
    model_path = os.path.join(dirname, model_filename or "__model__")
    with open(model_path, "wb") as f:
        f.write(inference_program.serialize_to_string())
    save_persistables(executor, dirname, inference_program, params_filename)
    return [t.name for t in target_vars]


def load_inference_model(dirname, executor, model_filename=None, params_filename=None, pserver_endpoints=None):
    model_path = os.path.join(dirname, model_filename or "__model__")
    with open(model_path, "rb") as f:
        program = Program.parse_from_string(f.read())
    load_persistables(executor, dirname, program, params_filename)
    gb = program.global_block()
    feed_names = [None] * sum(1 for op in gb.ops if op.type == "feed")
    fetch_vars = [None] * sum(1 for op in gb.ops if op.type == "fetch")
    for op in gb.ops:
        if op.type == "feed":
            feed_names[op.attrs["col"]] = op.output("Out")[0]
        elif op.type == "fetch":
            fetch_vars[op.attrs["col"]] = gb.var(op.input("X")[0])
    return program, feed_names, fetch_vars


def get_parameter_value(para, executor):
    return global_scope().find_var(para.name).get_tensor().numpy()


def get_parameter_value_by_name(name, executor, program=None):
    if program is None:
        program = default_main_program()
    return get_parameter_value(program.global_block().var(name), executor)
