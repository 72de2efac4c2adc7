"""Seq2seq decoder helpers (reference: python/paddle/fluid/contrib/decoder/
beam_search_decoder.py -- ``InitState``, ``StateCell``, ``TrainingDecoder``,
``BeamSearchDecoder``).

A :class:`StateCell` describes one decoding step as a function of named inputs and
named states (``state_updater``); the same cell runs inside

  * :class:`TrainingDecoder` -- teacher forcing over the target sequence, built on
    :class:`~paddle_amd.fluid.layers.DynamicRNN` (states are RNN memories, so the
    whole decoder trains through ``while_grad``);
  * :class:`BeamSearchDecoder` -- generation: a ``While`` loop whose states, ids and
    scores live in tensor arrays indexed by the step counter; every step expands
    the states to the live beams, scores the vocabulary, keeps ``topk_size``
    candidates per beam and lets the ``beam_search`` op select ``beam_size`` per
    source; decoding stops at ``max_len`` or when every beam has emitted ``end_id``.
"""
from __future__ import annotations

import contextlib

from ...framework import core
from .. import layers
from ..framework import Variable


class _DecoderType:
    TRAINING = 1
    BEAM_SEARCH = 2


class InitState:
    """Initial value of a decoder state: ``init`` directly, or a constant of
    ``shape`` filled with ``value`` whose batch size follows ``init_boot``."""

    def __init__(self, init=None, shape=None, value=0.0, init_boot=None, need_reorder=False, dtype="float32"):
        if init is not None:
            self._init = init
        elif init_boot is None:
            raise ValueError("init_boot must be provided to infer the shape of InitState .")
        else:
            self._init = layers.fill_constant_batch_size_like(input=init_boot, value=value, shape=shape,
                                                              dtype=dtype)
        self._shape = shape
        self._value = value
        self._need_reorder = need_reorder
        self._dtype = dtype

    @property
    def value(self):
        return self._init

    @property
    def need_reorder(self):
        return self._need_reorder


class _MemoryState:
    """State held as a DynamicRNN memory (training)."""

    def __init__(self, state_name, rnn_obj, init_state):
        self._state_name = state_name
        self._rnn_obj = rnn_obj
        self._state_mem = self._rnn_obj.memory(init=init_state.value, need_reorder=init_state.need_reorder)

    def get_state(self):
        return self._state_mem

    def update_state(self, state):
        self._rnn_obj.update_memory(self._state_mem, state)


class _ArrayState:
    """State held in a tensor array indexed by the decoder's step counter (generation)."""

    def __init__(self, state_name, decoder, init_state):
        self._state_name = state_name
        self._decoder = decoder
        self._state_read = decoder.read_array(init=init_state.value)

    def get_state(self):
        return self._state_read

    def update_state(self, state):
        self._decoder.update_array(self._state_read, state)


class StateCell:
    """One decoding step: named ``inputs`` (dict name -> Variable or None) and
    ``states`` (dict name -> InitState); ``out_state`` names the state exposed as
    the cell's output."""

    def __init__(self, inputs, states, out_state, name=None):
        self._helper_name = name or "state_cell"
        self._inputs = dict(inputs)
        self._init_states = dict(states)
        self._state_names = list(states.keys())
        if out_state not in self._init_states:
            raise ValueError("out_state must be one state in states")
        self._out_state = out_state
        self._cur_states = {}
        self._states_holder = {}
        self._cur_decoder_obj = None
        self._in_decoder = False
        self._state_updater = None
        self._switched_decoder = False

    # --------------------------------------------------------------- decoder hooks
    def _enter_decoder(self, decoder_obj):
        if self._in_decoder or self._cur_decoder_obj is not None:
            raise ValueError("StateCell has already entered a decoder.")
        self._in_decoder = True
        self._cur_decoder_obj = decoder_obj
        self._switched_decoder = False

    def _leave_decoder(self, decoder_obj):
        if not self._in_decoder:
            raise ValueError("StateCell not in decoder, invalid leaving operation.")
        if self._cur_decoder_obj != decoder_obj:
            raise ValueError("Inconsistent decoder object in StateCell.")
        self._in_decoder = False
        self._cur_decoder_obj = None
        self._switched_decoder = False

    def _switch_decoder(self):
        """Materialise the states inside the current decoder's step block."""
        if not self._in_decoder:
            raise ValueError("StateCell must be enter a decoder.")
        if self._switched_decoder:
            raise ValueError("StateCell already done switching.")
        dec = self._cur_decoder_obj
        for name in self._state_names:
            init = self._init_states[name]
            if dec.type == _DecoderType.TRAINING:
                holder = _MemoryState(name, dec.dynamic_rnn, init)
            else:
                holder = _ArrayState(name, dec, init)
            self._states_holder[name] = {id(dec): holder}
            self._cur_states[name] = holder.get_state()
        self._switched_decoder = True

    def _holder(self, name):
        return self._states_holder[name][id(self._cur_decoder_obj)]

    # --------------------------------------------------------------- public API
    def get_state(self, state_name):
        if self._in_decoder and not self._switched_decoder:
            self._switch_decoder()
        if state_name not in self._cur_states:
            raise ValueError(f"Unknown state {state_name}. Please make sure _switch_decoder() invoked.")
        return self._cur_states[state_name]

    def get_input(self, input_name):
        if input_name not in self._inputs or self._inputs[input_name] is None:
            raise ValueError(f"Invalid input {input_name}.")
        return self._inputs[input_name]

    def set_state(self, state_name, state_value):
        self._cur_states[state_name] = state_value

    def state_updater(self, updater):
        self._state_updater = updater

        def _decorator(state_cell):
            if state_cell == self:
                raise TypeError("Updater should only accept a StateCell object as argument.")
            updater(state_cell)

        return _decorator

    def compute_state(self, inputs):
        if self._in_decoder and not self._switched_decoder:
            self._switch_decoder()
        for name, value in inputs.items():
            if name not in self._inputs:
                raise ValueError(f"Unknown input {name}. Please make sure {name} in input place holder.")
            self._inputs[name] = value
        self._state_updater(self)

    def update_states(self):
        if self._in_decoder and not self._switched_decoder:
            self._switch_decoder()
        for name, holder in self._states_holder.items():
            h = holder[id(self._cur_decoder_obj)]
            h.update_state(self._cur_states[name])

    def out_state(self):
        return self._cur_states[self._out_state]


class TrainingDecoder:
    """Teacher-forced decoder over target sequences (a DynamicRNN underneath)."""

    BEFORE_DECODER, IN_DECODER, AFTER_DECODER = 0, 1, 2

    def __init__(self, state_cell, name=None):
        self._status = TrainingDecoder.BEFORE_DECODER
        self._dynamic_rnn = layers.DynamicRNN()
        self._type = _DecoderType.TRAINING
        self._state_cell = state_cell
        self._state_cell._enter_decoder(self)

    @contextlib.contextmanager
    def block(self):
        if self._status != TrainingDecoder.BEFORE_DECODER:
            raise ValueError("decoder.block() can only be invoked once")
        self._status = TrainingDecoder.IN_DECODER
        with self._dynamic_rnn.block():
            yield
        self._status = TrainingDecoder.AFTER_DECODER
        self._state_cell._leave_decoder(self)

    @property
    def state_cell(self):
        self._assert_in_decoder_block("state_cell")
        return self._state_cell

    @property
    def dynamic_rnn(self):
        return self._dynamic_rnn

    @property
    def type(self):
        return self._type

    def step_input(self, x):
        self._assert_in_decoder_block("step_input")
        return self._dynamic_rnn.step_input(x)

    def static_input(self, x):
        self._assert_in_decoder_block("static_input")
        return self._dynamic_rnn.static_input(x)

    def __call__(self, *args, **kwargs):
        if self._status != TrainingDecoder.AFTER_DECODER:
            raise ValueError("Output of training decoder can only be visited outside the block.")
        return self._dynamic_rnn(*args, **kwargs)

    def output(self, *outputs):
        self._assert_in_decoder_block("output")
        self._dynamic_rnn.output(*outputs)

    def _assert_in_decoder_block(self, method):
        if self._status != TrainingDecoder.IN_DECODER:
            raise ValueError(f"{method} should be invoked inside block of TrainingDecoder object.")


class BeamSearchDecoder:
    """Beam-search generation with a StateCell (see the module docstring)."""

    BEFORE_BEAM_SEARCH_DECODER, IN_BEAM_SEARCH_DECODER, AFTER_BEAM_SEARCH_DECODER = 0, 1, 2

    def __init__(self, state_cell, init_ids, init_scores, target_dict_dim, word_dim, input_var_dict=None,
                 topk_size=50, sparse_emb=True, max_len=100, beam_size=1, end_id=1, name=None):
        self._type = _DecoderType.BEAM_SEARCH
        self._status = BeamSearchDecoder.BEFORE_BEAM_SEARCH_DECODER
        self._max_len = layers.fill_constant(shape=[1], dtype="int64", value=max_len)
        self._zero_idx = layers.fill_constant(shape=[1], dtype="int64", value=0)
        self._counter = layers.fill_constant(shape=[1], dtype="int64", value=0)
        self._counter.stop_gradient = True
        self._cond = layers.less_than(x=self._counter, y=self._max_len)
        self._while_op = layers.While(self._cond)
        self._state_cell = state_cell
        self._state_cell._enter_decoder(self)
        self._init_ids = init_ids
        self._init_scores = init_scores
        self._target_dict_dim = target_dict_dim
        self._topk_size = topk_size
        self._sparse_emb = sparse_emb
        self._word_dim = word_dim
        self._input_var_dict = dict(input_var_dict or {})
        self._array_dict = {}
        self._array_link = []
        self._ids_array = None
        self._scores_array = None
        self._beam_size = beam_size
        self._end_id = end_id

    @property
    def type(self):
        return self._type

    @property
    def state_cell(self):
        self._assert_in_decoder_block("state_cell")
        return self._state_cell

    @contextlib.contextmanager
    def block(self):
        if self._status != BeamSearchDecoder.BEFORE_BEAM_SEARCH_DECODER:
            raise ValueError("block() can only be invoke once.")
        self._status = BeamSearchDecoder.IN_BEAM_SEARCH_DECODER
        with self._while_op.block():
            yield
            layers.increment(x=self._counter, value=1.0, in_place=True)
            for value, array in self._array_link:
                layers.array_write(x=value, i=self._counter, array=array)
            in_len = layers.less_than(x=self._counter, y=self._max_len)
            layers.assign(layers.logical_and(x=self._cond, y=in_len), self._cond)
        self._status = BeamSearchDecoder.AFTER_BEAM_SEARCH_DECODER
        self._state_cell._leave_decoder(self)

    def early_stop(self):
        """Stop decoding after this step (sets the loop condition to False)."""
        layers.fill_constant(shape=[1], dtype="bool", value=0, out=self._cond)

    def decode(self):
        """Default step: embed the previous ids, run the state cell on the states
        expanded to the live beams, score the vocabulary, keep top-k and select."""
        with self.block():
            prev_ids = self.read_array(init=self._init_ids, is_ids=True)
            prev_scores = self.read_array(init=self._init_scores, is_scores=True)
            prev_ids_embedding = layers.embedding(input=prev_ids, size=[self._target_dict_dim, self._word_dim],
                                                  dtype="float32", is_sparse=self._sparse_emb)
            feed_dict, update_dict = {}, {}
            for name, init_var in self._input_var_dict.items():
                if name not in self._state_cell._inputs:
                    raise ValueError(f"Variable {name} not found in StateCell!")
                read_var = self.read_array(init=init_var)
                update_dict[name] = read_var
                feed_dict[name] = layers.sequence_expand(read_var, prev_scores)
            for state_str in self._state_cell._state_names:
                prev_state = self._state_cell.get_state(state_str)
                self._state_cell.set_state(state_str, layers.sequence_expand(prev_state, prev_scores))
            for name in self._state_cell._inputs:
                if name not in feed_dict:
                    feed_dict[name] = prev_ids_embedding
            self._state_cell.compute_state(inputs=feed_dict)
            current_state = self._state_cell.out_state()
            current_state_with_lod = layers.lod_reset(x=current_state, y=prev_scores)
            scores = layers.fc(input=current_state_with_lod, size=self._target_dict_dim, act="softmax")
            topk_scores, topk_indices = layers.topk(scores, k=self._topk_size)
            accu_scores = layers.elementwise_add(x=layers.log(x=topk_scores),
                                                 y=layers.reshape(prev_scores, shape=[-1]), axis=0)
            selected_ids, selected_scores = layers.beam_search(prev_ids, prev_scores, topk_indices, accu_scores,
                                                               self._beam_size, end_id=self._end_id, level=0)
            with layers.Switch() as switch:
                with switch.case(layers.is_empty(selected_ids)):
                    self.early_stop()
                with switch.default():
                    self._state_cell.update_states()
                    self.update_array(prev_ids, selected_ids)
                    self.update_array(prev_scores, selected_scores)
                    for name, var_to_update in update_dict.items():
                        self.update_array(var_to_update, feed_dict[name])

    def read_array(self, init, is_ids=False, is_scores=False):
        """Tensor array seeded with ``init`` at step 0; returns its element at the
        current step (inside the block)."""
        self._assert_in_decoder_block("read_array")
        if is_ids and is_scores:
            raise ValueError("Shouldn't mark current array be ids array and scores array at the same time.")
        if not isinstance(init, Variable):
            raise TypeError("The input argument `init` must be a Variable.")
        prog = init.block.program
        parent = prog.block(prog.current_block().parent_idx)
        array = parent.create_var(name=f"{init.name}_decoder_array", type=core.VT.LOD_TENSOR_ARRAY,
                                  dtype=init.dtype, shape=init.shape)
        parent.append_op(type="write_to_array", inputs={"X": [init], "I": [self._zero_idx]},
                         outputs={"Out": [array]})
        if is_ids:
            self._ids_array = array
        elif is_scores:
            self._scores_array = array
        read_value = layers.array_read(array=array, i=self._counter)
        read_value.shape = init.shape
        read_value.lod_level = init.lod_level
        self._array_dict[read_value.name] = array
        return read_value

    def update_array(self, array, value):
        """Write ``value`` as the next step's element of the array ``array`` was read from."""
        self._assert_in_decoder_block("update_array")
        if not isinstance(array, Variable) or not isinstance(value, Variable):
            raise TypeError("The input argument `array` and `value` must be Variables.")
        array_var = self._array_dict.get(array.name)
        if array_var is None:
            raise ValueError("Please invoke read_array before update_array.")
        self._array_link.append((value, array_var))

    def __call__(self):
        if self._status != BeamSearchDecoder.AFTER_BEAM_SEARCH_DECODER:
            raise ValueError("Output of BeamSearchDecoder object can only be visited outside the block.")
        return layers.beam_search_decode(ids=self._ids_array, scores=self._scores_array, beam_size=self._beam_size,
                                         end_id=self._end_id)

    def _assert_in_decoder_block(self, method):
        if self._status != BeamSearchDecoder.IN_BEAM_SEARCH_DECODER:
            raise ValueError(f"{method} should be invoked inside block of BeamSearchDecoder object.")
