from pytorchrec_amd.model.layer.Dense import Dense
from pytorchrec_amd.model.layer.MLP import MLP
