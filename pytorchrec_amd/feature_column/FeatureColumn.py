"""Feature column base (torchrec/feature_column/FeatureColumn.py:10-26)."""
from abc import ABC, abstractmethod
from typing import Any, Dict

from torch import Tensor


class FeatureColumn(ABC):
    """Base of all feature columns: a name-keyed view into the batch dict plus a
    free-form info dict (set_info/get_info, FeatureColumn.py:13-22)."""

    def __init__(self):
        self._info: Dict[str, Any] = {}

    def set_info(self, key: str, value: Any) -> None:
        self._info[key] = value

    def get_info(self) -> Dict:
        return self._info

    @abstractmethod
    def get_feature_data(self, *args, **kwargs) -> Tensor:
        """Extract this column's tensor from a batch."""
