"""pytorchrec_amd — MI355X-native embedding-lookup + feature-interaction hot path.

Drop-in behind the ``torchrec.feature_column`` / ``torchrec.model`` API of
Troublem1/PyTorchRec: ``pytorchrec_amd.feature_column`` and
``pytorchrec_amd.model`` mirror those packages; on a GPU every embedding /
interaction op runs in hand-written gfx950 HIP kernels (``libmrec.so``, C ABI in
``include/mrec.h``) and fails loudly if the library is missing.
"""
__version__ = "0.1.0"
