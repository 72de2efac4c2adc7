"""v2 topology (reference v2/topology.py): the data layers and the Fluid program a
set of output layers depends on."""
from ._core import STATE


class Topology:
    def __init__(self, layers, extra_layers=None):
        self.layers = layers if isinstance(layers, (list, tuple)) else [layers]
        self.extra_layers = extra_layers or []

    def proto(self):
        return STATE["main"]

    def data_layers(self):
        return dict(STATE["data"])

    def data_type(self):
        return list(STATE["data"].items())
