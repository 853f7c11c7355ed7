"""Declarative CLI argument (torchrec/utils/argument/ArgumentDescription.py:19-107)."""
import argparse
from argparse import ArgumentParser
from typing import Any, Type


def str2bool(v):
    if v.lower() == "true":
        return True
    if v.lower() == "false":
        return False
    raise argparse.ArgumentTypeError("Unsupported value encountered.")


class ArgumentDescription:
    """Name, type (str/int/float/bool), default, legal values and open/closed
    numeric bounds of one argument; ``check_value`` asserts them."""
    _types = {str, int, float, bool}
    _number_types = {int, float}

    def __init__(self, name: str, type_: Type, help_info: str, is_logged: bool = True,
                 default_value=None, legal_value_list=None, lower_open_bound=None,
                 lower_closed_bound=None, upper_open_bound=None, upper_closed_bound=None):
        assert type_ in self._types
        if default_value is not None:
            assert isinstance(default_value, type_)
        if legal_value_list:
            for v in legal_value_list:
                assert isinstance(v, type_)
            lower_open_bound = lower_closed_bound = upper_open_bound = upper_closed_bound = None
        bounds = (lower_open_bound, lower_closed_bound, upper_open_bound, upper_closed_bound)
        if any(b is not None for b in bounds):
            assert type_ in self._number_types
            for b in bounds:
                assert b is None or isinstance(b, (int, float))
        self.name = name
        self.type = type_
        self.help_info = help_info
        self.is_logged = is_logged
        self.default_value = default_value
        self.legal_value_list = legal_value_list
        self.lower_open_bound = lower_open_bound
        self.lower_closed_bound = lower_closed_bound
        self.upper_open_bound = upper_open_bound
        self.upper_closed_bound = upper_closed_bound
        if default_value is not None:
            self.check_value(default_value)

    def check_value(self, value: Any) -> None:
        if self.legal_value_list:
            assert value in self.legal_value_list, f"{self.name}={value!r} not in {self.legal_value_list}"
            return
        if self.lower_open_bound is not None:
            assert self.lower_open_bound < value, f"{self.name}={value} <= {self.lower_open_bound}"
        if self.lower_closed_bound is not None:
            assert self.lower_closed_bound <= value, f"{self.name}={value} < {self.lower_closed_bound}"
        if self.upper_open_bound is not None:
            assert value < self.upper_open_bound, f"{self.name}={value} >= {self.upper_open_bound}"
        if self.upper_closed_bound is not None:
            assert value <= self.upper_closed_bound, f"{self.name}={value} > {self.upper_closed_bound}"

    def add_argument_into_argparser(self, parser: ArgumentParser):
        parser.add_argument("--" + self.name, type=str2bool if self.type == bool else self.type,
                            help=self.help_info, default=self.default_value,
                            required=self.default_value is None)
