"""Utilities mirrored from ``torchrec.utils`` that the model plug-in contract needs."""
from pytorchrec_amd.utils.global_utils import set_torch_seed
from pytorchrec_amd.utils.data_structure import tensor_to_device, map_structure
