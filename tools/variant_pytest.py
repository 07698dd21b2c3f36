"""pytest against a compile-time variant of the library (tools/build_variants.py):
DPFT_LIB=tools/libs/libdpft_<name>.so python tools/variant_pytest.py tests -m gpu -q"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_prob_feature_track_amd import _native
if os.environ.get("DPFT_LIB"):
    _native.LIB_PATH = os.path.abspath(os.environ["DPFT_LIB"])
import pytest
sys.exit(pytest.main(sys.argv[1:]))
