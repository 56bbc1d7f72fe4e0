"""Host helpers of shipping/util.py (the kernel restates both in its step)."""
import numpy as np


def calculate_euclidean_distance(start, end):
    """np.sqrt of the integer sum of squares (shipping/util.py:3-4)."""
    return np.sqrt((end[0] - start[0]) ** 2 + (end[1] - start[1]) ** 2)


def normalize(raw, max, min):  # noqa: A002 - the reference's parameter names
    """(raw - min) / (max - min), or raw / max when min == 0 (shipping/util.py:6-10)."""
    if min == 0:
        return raw / max
    return (raw - min) / (max - min)
