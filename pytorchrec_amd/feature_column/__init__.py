"""Feature columns — mirror of ``torchrec.feature_column`` (the API the hot path
stays drop-in behind)."""
from pytorchrec_amd.feature_column.FeatureColumn import FeatureColumn
from pytorchrec_amd.feature_column.CategoricalColumn import CategoricalColumn
from pytorchrec_amd.feature_column.CategoricalColumnWithIdentity import CategoricalColumnWithIdentity
from pytorchrec_amd.feature_column.CrossedColumn import CrossedColumn
from pytorchrec_amd.feature_column.DenseColumn import DenseColumn
from pytorchrec_amd.feature_column.NormalizationMode import NormalizationMode
from pytorchrec_amd.feature_column.NumericColumn import NumericColumn

__all__ = ["FeatureColumn", "CategoricalColumn", "CategoricalColumnWithIdentity", "CrossedColumn",
           "DenseColumn", "NormalizationMode", "NumericColumn"]
