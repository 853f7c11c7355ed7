"""Numeric normalisation modes (torchrec/feature_column/NormalizationMode.py:8-12)."""
from enum import Enum, unique


@unique
class NormalizationMode(Enum):
    NOP = "nop"
    MAX_MIN = "max_min"
    Z_SCORE = "z_score"
