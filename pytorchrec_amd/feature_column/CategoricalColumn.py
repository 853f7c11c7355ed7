"""Categorical column base (torchrec/feature_column/CategoricalColumn.py:9-14)."""
from abc import ABC

from pytorchrec_amd.feature_column.FeatureColumn import FeatureColumn


class CategoricalColumn(FeatureColumn, ABC):
    """A column of integer categories in [0, category_num) — the row count of the
    embedding table it indexes."""

    def __init__(self, category_num: int):
        super().__init__()
        self.category_num = category_num
