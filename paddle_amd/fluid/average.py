"""WeightedAverage (python/paddle/fluid/average.py)."""
import numpy as np

__all__ = ["WeightedAverage"]


class WeightedAverage:
    def __init__(self):
        self.reset()

    def reset(self):
        self.numerator = None
        self.denominator = None

    def add(self, value, weight):
        value = np.asarray(value, dtype="float64")
        if self.numerator is None:
            self.numerator = value * weight
            self.denominator = weight
        else:
            self.numerator += value * weight
            self.denominator += weight

    def eval(self):
        if self.numerator is None:
            raise ValueError("There is no data to be averaged in WeightedAverage.")
        return self.numerator / self.denominator
