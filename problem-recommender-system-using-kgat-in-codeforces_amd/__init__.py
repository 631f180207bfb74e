"""MI355X-native KGAT / NFM training + scoring path (gfx950 HIP kernels behind a C-ABI).

Drop-in for the reference's src/model/KGAT/model.py and src/model/NFM/model.py
module API.  Import with ``importlib.import_module(
"problem-recommender-system-using-kgat-in-codeforces_amd")`` (the directory
name is not a Python identifier).
"""
from .graph import DeviceGraph, GraphLayout, build_layout, synthetic_ckg  # noqa: F401
from . import evaluation  # noqa: F401
from .model import KGAT, KGATArgs, KGATMode  # noqa: F401
from .nfm import NFM, NFMArgs, NFMBatch, NFMBatcher, NFMMode  # noqa: F401

__all__ = ["evaluation", "KGAT", "KGATArgs", "KGATMode", "NFM", "NFMArgs", "NFMBatch", "NFMBatcher", "NFMMode", "DeviceGraph", "GraphLayout", "build_layout",
           "synthetic_ckg"]
