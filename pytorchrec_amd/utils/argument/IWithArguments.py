"""Argument-declaring interface (torchrec/utils/argument/IWithArguments.py:10-28)."""
from abc import ABC
from typing import Any, Dict, List

from pytorchrec_amd.utils.argument.ArgumentDescription import ArgumentDescription


class IWithArguments(ABC):
    """Classes declare their CLI arguments and validate values against them."""

    @classmethod
    def get_argument_descriptions(cls) -> List[ArgumentDescription]:
        return []

    @classmethod
    def check_argument_values(cls, arguments: Dict[str, Any]) -> None:
        for d in cls.get_argument_descriptions():
            d.check_value(arguments[d.name])
