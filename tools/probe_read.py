"""Measured HBM read ceiling of the diagnostic streaming read (dpft_read_probe) at two
buffer sizes; DPFT_LIB selects a variant build (tools/build_variants.py)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from deep_prob_feature_track_amd import _native as N  # noqa: E402

if os.environ.get("DPFT_LIB"):
    N.LIB_PATH = os.path.abspath(os.environ["DPFT_LIB"])
import bench  # noqa: E402

dev = torch.device("cuda:0")
for n in (668467200, 2 << 30):
    print(os.path.basename(N.LIB_PATH), n, round(bench.read_peak_gbs(dev, n, reps=20)), flush=True)
