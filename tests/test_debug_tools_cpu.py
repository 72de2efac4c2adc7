"""Debug / trace tooling: program pretty-printer and block graph (fluid/debugger.py),
net_drawer.draw_graph, the profiler's profile dump and tools/timeline.py's Chrome
trace (reference: python/paddle/fluid/debugger.py, net_drawer.py, tools/timeline.py)."""
import json
import os
import sys

import numpy as np

import paddle_amd.fluid as fluid
from paddle_amd.fluid import debugger, net_drawer


def _prog():
    main, st = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, st):
        x = fluid.layers.data("x", [8])
        y = fluid.layers.fc(x, 4, act="relu")
        loss = fluid.layers.mean(y)
        fluid.optimizer.SGD(0.1).minimize(loss)
    return main, st, loss


def test_pprint_program_codes_hides_backward_by_default():
    main, _, _ = _prog()
    txt = debugger.pprint_program_codes(main)
    assert "// block-0" in txt and "= mul(X=x, Y=fc_" in txt
    assert "[persistable]" in txt
    assert "_grad(" not in txt and "@GRAD" not in txt
    full = debugger.pprint_program_codes(main, show_backward=True)
    assert "mul_grad(" in full and "sgd(" in full


def test_draw_block_graphviz_and_net_drawer(tmp_path):
    main, st, _ = _prog()
    dot = debugger.draw_block_graphviz(main.global_block(), highlights=[r"fc_\d+\.w_.*"], path=str(tmp_path / "b.dot"))
    assert dot.startswith("digraph") and "color=red" in dot and os.path.getsize(tmp_path / "b.dot") > 0
    g = net_drawer.draw_graph(st, main, filename=str(tmp_path / "n.dot"))
    assert "cluster_startup" in g and "cluster_main" in g and '"mul"' in g


def test_profiler_profile_and_timeline(tmp_path):
    main, st, loss = _prog()
    exe = fluid.Executor(fluid.CPUPlace())
    scope = fluid.Scope()
    prof_path = str(tmp_path / "profile")
    with fluid.scope_guard(scope):
        exe.run(st)
        with fluid.profiler.profiler("CPU", sorted_key="total", profile_path=prof_path):
            for _ in range(3):
                exe.run(main, feed={"x": np.random.rand(4, 8).astype("float32")}, fetch_list=[loss])
    prof = json.load(open(prof_path))
    names = {e["name"] for e in prof["events"]}
    assert {"mul", "relu", "sgd"} <= names and all(e["end_ns"] >= e["start_ns"] for e in prof["events"])
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import timeline

    out = timeline.main(["--profile_path", f"t0={prof_path},t1={prof_path}", "--timeline_path",
                         str(tmp_path / "tl.json")])
    tr = json.load(open(out))["traceEvents"]
    procs = {e["args"]["name"] for e in tr if e["ph"] == "M"}
    assert {"t0:cpu:block:0", "t1:cpu:block:0"} <= procs
    assert sum(1 for e in tr if e["ph"] == "X" and e["name"] == "mul") == 6
