"""v2 input types (reference v2/data_type.py over trainer/PyDataProvider2.py)."""
from dataclasses import dataclass


@dataclass(frozen=True)
class InputType:
    dim: int
    seq_type: int  # 0 no sequence, 1 sequence
    kind: str      # "dense" | "index"


def dense_vector(dim):
    return InputType(int(dim), 0, "dense")


def dense_vector_sequence(dim):
    return InputType(int(dim), 1, "dense")


def integer_value(value_range):
    return InputType(int(value_range), 0, "index")


def integer_value_sequence(value_range):
    return InputType(int(value_range), 1, "index")


dense_array = dense_vector
