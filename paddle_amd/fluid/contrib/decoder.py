"""Seq2seq decoder helpers: ``InitState``, ``StateCell``, ``TrainingDecoder``,
``BeamSearchDecoder`` (API of python/paddle/fluid/contrib/decoder/
beam_search_decoder.py; written from the documented behaviour).

Design:

* a :class:`StateCell` is a step function over named inputs and named states; it
  does not know where its states live.  Each decoder supplies a *state backend*
  through ``_new_state_slot(init)``: the training decoder backs a state with a
  DynamicRNN memory (so the whole decoder trains through ``while_grad``), the
  beam-search decoder with a tensor array indexed by the step counter;
* both decoders share :class:`_PhasedBlock`, which enforces the
  before / inside / after life cycle of their single ``block()``;
* beam search per step: expand the states and extra inputs to the live beams
  (``sequence_expand`` over the previous scores' LoD), run the cell, score the
  vocabulary, keep ``topk_size`` candidates per beam, let ``beam_search`` select
  ``beam_size`` per source, and stop when nothing survives or at ``max_len``.
"""
from __future__ import annotations

import contextlib

from ...framework import core
from .. import layers
from ..framework import Variable

_BEFORE, _INSIDE, _AFTER = "before", "inside", "after"


class InitState:
    """Initial value of one decoder state.

    Either ``init`` (a Variable) is used as is, or a ``shape``-shaped constant
    ``value`` is created whose batch dimension follows ``init_boot``.
    ``need_reorder``: the state is reordered with the beams / sorted sequences."""

    def __init__(self, init=None, shape=None, value=0.0, init_boot=None, need_reorder=False, dtype="float32"):
        if init is None:
            if init_boot is None:
                raise ValueError("InitState needs either `init` or `init_boot` (to size the batch)")
            init = layers.fill_constant_batch_size_like(input=init_boot, value=value, shape=shape, dtype=dtype)
        self._var = init
        self._reorder = bool(need_reorder)
        self._shape, self._fill, self._dtype = shape, value, dtype

    @property
    def value(self):
        return self._var

    @property
    def need_reorder(self):
        return self._reorder


class _RnnMemorySlot:
    """A state kept as a DynamicRNN memory (teacher-forced training)."""

    def __init__(self, rnn, init):
        self._rnn = rnn
        self._mem = rnn.memory(init=init.value, need_reorder=init.need_reorder)

    def read(self):
        return self._mem

    def write(self, value):
        self._rnn.update_memory(self._mem, value)


class _ArraySlot:
    """A state kept in a step-indexed tensor array (generation)."""

    def __init__(self, decoder, init):
        self._decoder = decoder
        self._cur = decoder.read_array(init=init.value)

    def read(self):
        return self._cur

    def write(self, value):
        self._decoder.update_array(self._cur, value)


class StateCell:
    """Named inputs (dict name -> Variable or None) and named states (dict name ->
    InitState); ``out_state`` names the state returned by :meth:`out_state`.
    The step function is registered with :meth:`state_updater`."""

    def __init__(self, inputs, states, out_state, name=None):
        if out_state not in states:
            raise ValueError(f"out_state {out_state!r} is not one of the states {list(states)}")
        self._name = name or "state_cell"
        self._inputs = dict(inputs)
        self._inits = dict(states)
        self._state_names = list(states)
        self._out_name = out_state
        self._updater = None
        self._owner = None     # decoder currently using this cell
        self._slots = None     # name -> state backend, created on first use inside a block
        self._current = {}     # name -> Variable for this step

    # -- decoder protocol ---------------------------------------------------
    def _attach(self, decoder):
        if self._owner is not None:
            raise ValueError("this StateCell is already used by another decoder")
        self._owner = decoder
        self._slots = None

    def _detach(self, decoder):
        if self._owner is not decoder:
            raise ValueError("StateCell detached from a decoder it was not attached to")
        self._owner = None
        self._slots = None

    def _materialize(self):
        if self._owner is None:
            raise ValueError("StateCell states are only available inside a decoder block")
        if self._slots is None:
            self._slots = {n: self._owner._new_state_slot(self._inits[n]) for n in self._state_names}
            self._current = {n: slot.read() for n, slot in self._slots.items()}

    # -- public API -----------------------------------------------------------
    def get_state(self, state_name):
        self._materialize()
        try:
            return self._current[state_name]
        except KeyError:
            raise ValueError(f"StateCell has no state named {state_name!r}") from None

    def set_state(self, state_name, state_value):
        self._current[state_name] = state_value

    def get_input(self, input_name):
        v = self._inputs.get(input_name)
        if v is None:
            raise ValueError(f"StateCell input {input_name!r} is missing or not fed yet")
        return v

    def state_updater(self, updater):
        """Register ``updater(cell)``, the step function (usable as a decorator)."""
        self._updater = updater
        return updater

    def compute_state(self, inputs):
        self._materialize()
        unknown = [k for k in inputs if k not in self._inputs]
        if unknown:
            raise ValueError(f"StateCell got inputs it does not declare: {unknown}")
        self._inputs.update(inputs)
        if self._updater is None:
            raise ValueError("StateCell has no state updater; register one with state_updater()")
        self._updater(self)

    def update_states(self):
        self._materialize()
        for n, slot in self._slots.items():
            slot.write(self._current[n])

    def out_state(self):
        return self._current[self._out_name]


class _PhasedBlock:
    """before -> inside (exactly one ``block()``) -> after."""

    def _init_phase(self, cell):
        self._phase = _BEFORE
        self._state_cell = cell
        cell._attach(self)

    @contextlib.contextmanager
    def _phase_block(self, inner):
        if self._phase != _BEFORE:
            raise ValueError(f"{type(self).__name__}.block() may be entered only once")
        self._phase = _INSIDE
        with inner:
            yield
            self._on_block_end()
        self._phase = _AFTER
        self._state_cell._detach(self)

    def _on_block_end(self):
        pass

    def _require(self, phase, what):
        if self._phase != phase:
            where = "inside" if phase == _INSIDE else "after"
            raise ValueError(f"{type(self).__name__}.{what} is only valid {where} the decoder block")

    @property
    def state_cell(self):
        self._require(_INSIDE, "state_cell")
        return self._state_cell


class TrainingDecoder(_PhasedBlock):
    """Teacher-forced decoder over the target sequences (a DynamicRNN)."""

    def __init__(self, state_cell, name=None):
        self._rnn = layers.DynamicRNN()
        self._init_phase(state_cell)

    def block(self):
        return self._phase_block(self._rnn.block())

    def _new_state_slot(self, init):
        return _RnnMemorySlot(self._rnn, init)

    @property
    def dynamic_rnn(self):
        return self._rnn

    @property
    def type(self):
        return "training"

    def step_input(self, x):
        self._require(_INSIDE, "step_input")
        return self._rnn.step_input(x)

    def static_input(self, x):
        self._require(_INSIDE, "static_input")
        return self._rnn.static_input(x)

    def output(self, *outputs):
        self._require(_INSIDE, "output")
        self._rnn.output(*outputs)

    def __call__(self, *args, **kwargs):
        self._require(_AFTER, "__call__")
        return self._rnn(*args, **kwargs)


class BeamSearchDecoder(_PhasedBlock):
    """Beam-search generation driven by a StateCell (module docstring)."""

    def __init__(self, state_cell, init_ids, init_scores, target_dict_dim, word_dim, input_var_dict=None,
                 topk_size=50, sparse_emb=True, max_len=100, beam_size=1, end_id=1, name=None):
        self._step = layers.fill_constant(shape=[1], dtype="int64", value=0)
        self._step.stop_gradient = True
        self._first = layers.fill_constant(shape=[1], dtype="int64", value=0)
        self._limit = layers.fill_constant(shape=[1], dtype="int64", value=max_len)
        self._running = layers.less_than(x=self._step, y=self._limit)
        self._loop = layers.While(self._running)
        self._init_ids, self._init_scores = init_ids, init_scores
        self._vocab, self._word_dim = target_dict_dim, word_dim
        self._extra_inputs = dict(input_var_dict or {})
        self._topk, self._beam, self._end_id = topk_size, beam_size, end_id
        self._sparse_emb = sparse_emb
        self._arrays = {}         # name of the per-step read Variable -> its tensor array
        self._writes = []         # (value, array) committed at the end of every step
        self._ids_array = self._scores_array = None
        self._init_phase(state_cell)

    @property
    def type(self):
        return "beam_search"

    def block(self):
        return self._phase_block(self._loop.block())

    def _on_block_end(self):
        layers.increment(x=self._step, value=1.0, in_place=True)
        for value, array in self._writes:
            layers.array_write(x=value, i=self._step, array=array)
        more = layers.less_than(x=self._step, y=self._limit)
        layers.assign(layers.logical_and(x=self._running, y=more), self._running)

    def _new_state_slot(self, init):
        return _ArraySlot(self, init)

    def early_stop(self):
        """Make this step the last one."""
        layers.fill_constant(shape=[1], dtype="bool", value=0, out=self._running)

    # -- per-step tensor arrays ------------------------------------------------
    def read_array(self, init, is_ids=False, is_scores=False):
        """Create a tensor array holding ``init`` at step 0 and return its element
        for the current step."""
        self._require(_INSIDE, "read_array")
        if is_ids and is_scores:
            raise ValueError("an array cannot hold both the ids and the scores")
        if not isinstance(init, Variable):
            raise TypeError(f"read_array expects a Variable, got {type(init).__name__}")
        prog = init.block.program
        outer = prog.block(prog.current_block().parent_idx)
        array = outer.create_var(name=f"{init.name}_decoder_array", type=core.VT.LOD_TENSOR_ARRAY,
                                 dtype=init.dtype, shape=init.shape)
        outer.append_op(type="write_to_array", inputs={"X": [init], "I": [self._first]},
                        outputs={"Out": [array]})
        if is_ids:
            self._ids_array = array
        if is_scores:
            self._scores_array = array
        cur = layers.array_read(array=array, i=self._step)
        cur.shape, cur.lod_level = init.shape, init.lod_level
        self._arrays[cur.name] = array
        return cur

    def update_array(self, array, value):
        """Store ``value`` as the next step's element of the array ``array`` came from."""
        self._require(_INSIDE, "update_array")
        if not (isinstance(array, Variable) and isinstance(value, Variable)):
            raise TypeError("update_array expects Variables")
        target = self._arrays.get(array.name)
        if target is None:
            raise ValueError(f"{array.name} was not produced by read_array()")
        self._writes.append((value, target))

    # -- the default step ------------------------------------------------------
    def _beam_expand(self, var, beams):
        return layers.sequence_expand(var, beams)

    def _score(self, state, beams):
        state = layers.lod_reset(x=state, y=beams)
        probs = layers.fc(input=state, size=self._vocab, act="softmax")
        top_p, top_ids = layers.topk(probs, k=self._topk)
        total = layers.elementwise_add(x=layers.log(x=top_p), y=layers.reshape(beams, shape=[-1]), axis=0)
        return top_ids, total

    def decode(self):
        """Default generation step (module docstring); call instead of writing the
        loop body by hand."""
        with self.block():
            ids = self.read_array(init=self._init_ids, is_ids=True)
            scores = self.read_array(init=self._init_scores, is_scores=True)
            word = layers.embedding(input=ids, size=[self._vocab, self._word_dim], dtype="float32",
                                    is_sparse=self._sparse_emb)
            cell = self._state_cell
            carried, fed = {}, {}
            for name, init in self._extra_inputs.items():
                if name not in cell._inputs:
                    raise ValueError(f"input_var_dict entry {name!r} is not an input of the StateCell")
                carried[name] = self.read_array(init=init)
                fed[name] = self._beam_expand(carried[name], scores)
            for name in cell._state_names:
                cell.set_state(name, self._beam_expand(cell.get_state(name), scores))
            fed.update({name: word for name in cell._inputs if name not in fed})
            cell.compute_state(inputs=fed)
            top_ids, total = self._score(cell.out_state(), scores)
            new_ids, new_scores = layers.beam_search(ids, scores, top_ids, total, self._beam, end_id=self._end_id,
                                                     level=0)
            with layers.Switch() as sw:
                with sw.case(layers.is_empty(new_ids)):
                    self.early_stop()
                with sw.default():
                    cell.update_states()
                    self.update_array(ids, new_ids)
                    self.update_array(scores, new_scores)
                    for name, cur in carried.items():
                        self.update_array(cur, fed[name])

    def __call__(self):
        self._require(_AFTER, "__call__")
        return layers.beam_search_decode(ids=self._ids_array, scores=self._scores_array, beam_size=self._beam,
                                         end_id=self._end_id)
