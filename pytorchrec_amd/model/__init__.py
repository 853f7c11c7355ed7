"""Models — mirror of ``torchrec.model`` plus the CTR models of the hot path."""
from pytorchrec_amd.model.IModel import IModel
from pytorchrec_amd.model.DeepFM import FM, DeepFM
from pytorchrec_amd.model.DCNv2 import DCNv2
from pytorchrec_amd.model.DIN import DIN
from pytorchrec_amd.model.FunkSVD import FunkSVD
from pytorchrec_amd.model.models import get_model_type, model_name_list
