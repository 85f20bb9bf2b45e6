"""FastDepth evaluation metrics of src/GuideDepth/metrics.py on MI355X.

Result.evaluate (metrics.py:41-62) reduces output / target on the GPU with one
HIP pass (mde_eval_sums, every metric is a closed form of its sums) instead of
eleven ATen reductions; AverageMeter (:65-110) is host bookkeeping with the
reference's fields and averaging.
"""
from __future__ import annotations

import math

import numpy as np

from ..functional import eval_sums


# Result's fields in update()'s positional order (reference signature metrics.py:35-36).
# Error metrics are "lower is better" (worst = inf); the delta accuracies and the two
# timings are not (worst = 0).
_UPDATE_ORDER = ("irmse", "imae", "mse", "rmse", "rmse_log", "mae", "absrel", "lg10",
                 "delta1", "delta2", "delta3", "gpu_time", "data_time")
_WORST = {f: (0 if f.startswith("delta") or f.endswith("_time") else np.inf)
          for f in _UPDATE_ORDER}


class Result:
    """Same fields and methods as the reference's Result (metrics.py:14-62)."""

    def __init__(self):
        self.__dict__.update(dict.fromkeys(_UPDATE_ORDER, 0))

    def set_to_worst(self):
        self.__dict__.update(_WORST)

    def update(self, *values, **named):
        """update(irmse, imae, mse, rmse, rmse_log, mae, absrel, lg10, delta1, delta2, delta3,
        gpu_time, data_time) -- the reference's order, positional or by name."""
        given = dict(zip(_UPDATE_ORDER, values), **named)
        if len(values) > len(_UPDATE_ORDER) or set(given) != set(_UPDATE_ORDER):
            raise TypeError(f"update() needs exactly the fields {_UPDATE_ORDER}")
        self.__dict__.update(given)

    def evaluate(self, output, target):
        """All pixels of output / target (CUDA tensors of equal shape)."""
        s = [float(v) for v in eval_sums(output, target).tolist()]
        n = s[0]
        self.mse = s[4] / n
        self.rmse = math.sqrt(self.mse)
        self.mae = s[10] / n
        self.lg10 = s[9] / n
        self.rmse_log = math.sqrt(s[11] / n)
        self.absrel = s[6] / n
        self.delta1, self.delta2, self.delta3 = s[1] / n, s[2] / n, s[3] / n
        self.data_time = 0
        self.gpu_time = 0
        self.irmse = math.sqrt(s[13] / n)
        self.imae = s[12] / n


class AverageMeter:
    """Count-weighted running averages of Result fields (metrics.py:65-110).

    Two reference quirks: reset() reads self.sum_rmse_log before assigning it
    (metrics.py:74 -- the reference's constructor raises AttributeError; here
    it starts at 0), and average() hands mae / rmse_log to Result.update in
    swapped positions (:99-101 against update's signature :35) -- kept, so an
    average prints what the reference's would.
    """

    _FIELDS = ("irmse", "imae", "mse", "rmse", "mae", "rmse_log", "absrel", "lg10", "delta1",
               "delta2", "delta3")

    def __init__(self):
        self.reset()

    def reset(self):
        self.count = 0.0
        for f in self._FIELDS:
            setattr(self, "sum_" + f, 0)
        self.sum_data_time, self.sum_gpu_time = 0, 0

    def update(self, result, gpu_time, data_time, n=1):
        self.count += n
        for f in self._FIELDS:
            setattr(self, "sum_" + f, getattr(self, "sum_" + f) + n * getattr(result, f))
        self.sum_data_time += n * data_time
        self.sum_gpu_time += n * gpu_time

    def average(self):
        avg = Result()
        c = self.count
        avg.update(self.sum_irmse / c, self.sum_imae / c, self.sum_mse / c, self.sum_rmse / c,
                   self.sum_mae / c, self.sum_rmse_log / c, self.sum_absrel / c, self.sum_lg10 / c,
                   self.sum_delta1 / c, self.sum_delta2 / c, self.sum_delta3 / c,
                   self.sum_gpu_time / c, self.sum_data_time / c)
        return avg
