"""Dense column marker (torchrec/feature_column/DenseColumn.py)."""
from abc import ABC

from pytorchrec_amd.feature_column.FeatureColumn import FeatureColumn


class DenseColumn(FeatureColumn, ABC):
    """A column that can feed a deep network directly."""
