"""Probe: can a kernel store straight into torch's pinned host memory (zero-copy flag / count)?"""
import importlib
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
_lib = importlib.import_module("problem-recommender-system-using-kgat-in-codeforces_amd._lib")
g = importlib.import_module("problem-recommender-system-using-kgat-in-codeforces_amd.graph")
h = torch.zeros(64, dtype=torch.float32, pin_memory=True)
s = torch.cuda.current_stream().cuda_stream
_lib.call("kgat_fill_f32", h.data_ptr(), 64, 3.5, s)
torch.cuda.synchronize()
print("pinned write:", h[:4].tolist(), "ok" if float(h.sum()) == 3.5 * 64 else "FAILED")
