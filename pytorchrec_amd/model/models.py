"""Model registry — mirror of torchrec/model/models.py:8-30 (the plug-in point)."""
from typing import Dict, Type

from pytorchrec_amd.model.DCNv2 import DCNv2
from pytorchrec_amd.model.DeepFM import FM, DeepFM
from pytorchrec_amd.model.DIN import DIN
from pytorchrec_amd.model.FunkSVD import FunkSVD
from pytorchrec_amd.model.IModel import IModel

_model_classes: Dict[str, Type[IModel]] = {
    "funksvd": FunkSVD,
    "fm": FM,
    "deepfm": DeepFM,
    "dcnv2": DCNv2,
    "din": DIN,
}

model_name_list = _model_classes.keys()


def get_model_type(model_name: str) -> Type[IModel]:
    if (not isinstance(model_name, str)) or (model_name not in _model_classes):
        raise ValueError(f"model_name参数不合法: {model_name}")
    return _model_classes[model_name]
