"""The C-ABI library loads (no GPU needed) and exports every entry point include/dpft_ic.h declares."""
import os
import re

from deep_prob_feature_track_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "dpft_ic.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dpft_[a-z_]+)\s*\(", src)))


def test_header_declares_the_binding_surface():
    assert declared_functions() == sorted(N.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = N.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    assert L.dpft_version() == N.ABI_VERSION


def test_control_area_size_matches_the_library():
    """The Python side zeroes only the workspace's control prefix of private workspaces
    (ic.LevelCall): that prefix must be the library's kCtrlBytes, or stale completion
    counters would make the last-workgroup handshake misfire."""
    assert N.CTRL_BYTES == N.lib().dpft_preprocess_workspace_size()


def test_invalid_descriptor_is_rejected_without_device_work():
    import ctypes
    L = N.lib()
    bad = N.LevelDesc(0, 8, 1, 120, 160, 3, 0, 0.0)
    assert L.dpft_workspace_size(ctypes.byref(bad)) == 0
    rc = L.dpft_ic_solve_level(ctypes.byref(bad), None, None, None, None, None, None, 0, None)
    assert rc == -1 and b"bad shape" in L.dpft_last_error()
    cs = N.LevelDesc(1, 8, 3, 120, 160, 3, 0, 0.0)  # Cs must be 1 or C
    assert L.dpft_workspace_size(ctypes.byref(cs)) == 0


def test_group_descriptor_validation_without_device_work():
    """DPFT_GROUP(n): B a multiple of n, at most 32 batches (COMBINE_ICP too: per-batch
    depth1 extrema); n >= B (or 0) is one batch; n up to 2048 (a 12-bit field).  Checked by
    the descriptor validation every entry point runs."""
    import ctypes
    L = N.lib()
    G = lambda n: n << N.GROUP_SHIFT

    def ws(B, flags):
        return L.dpft_workspace_size(ctypes.byref(N.LevelDesc(B, 32, 1, 480, 640, 3, flags, 0.01)))
    base = N.REMOVE_TRU_SIGMA | N.FEATURES_C4
    assert ws(32, base | G(8)) > 0 and ws(32, base | G(8)) == ws(32, base)  # same workspace
    assert ws(8, base | G(8)) > 0 and ws(8, base | G(16)) > 0             # one batch
    assert ws(12, base | G(8)) == 0                                        # not a multiple
    assert b"DPFT_GROUP" in L.dpft_last_error()
    assert ws(64, base | G(1)) == 0                                        # 64 batches > 32
    assert ws(32, N.REMOVE_TRU_SIGMA | N.COMBINE_ICP | G(8)) > 0           # ICP: per-batch depth extrema
    assert ws(2048, base | G(256)) > 0 and ws(2048, base | G(256)) == ws(2048, base)  # 8 batches of 256
    assert ws(2048, base | G(1024)) > 0


def test_nchw_workspace_counts_the_entry_packs():
    """dpft_workspace_size for NCHW features that dpft_ic_solve_level / _pyramid pack to channel
    quads on entry (C % 16 == 0, one sigma plane, >= 2 iterations; include/dpft_ic.h): the
    channel-quad workspace plus two packed feature planes, each B C H W floats rounded up to 256
    bytes; where the solve does not pack (per-channel sigma, one iteration) nothing is added."""
    import ctypes
    L = N.lib()

    def ws(B, C, Cs, H, W, iters, flags):
        return L.dpft_workspace_size(ctypes.byref(N.LevelDesc(B, C, Cs, H, W, iters, flags, 0.0)))
    rnd = lambda n: (n + 255) // 256 * 256
    for B, C, H, W in ((8, 32, 480, 640), (1, 16, 120, 160), (3, 32, 61, 79)):
        c4 = ws(B, C, 1, H, W, 3, N.REMOVE_TRU_SIGMA | N.FEATURES_C4)
        nchw = ws(B, C, 1, H, W, 3, N.REMOVE_TRU_SIGMA)
        assert c4 > 0 and nchw == c4 + 2 * rnd(B * C * H * W * 4), (B, C, H, W)
    assert 0 < ws(2, 8, 1, 120, 160, 3, 0) == ws(2, 8, 1, 120, 160, 3, N.FEATURES_C4)   # C % 16 != 0: no pack
    assert 0 < ws(2, 32, 1, 120, 160, 1, 0) == ws(2, 32, 1, 120, 160, 1, N.FEATURES_C4)  # one iteration: no pack
    assert 0 < ws(2, 32, 32, 120, 160, 3, 0)  # per-channel sigma: the NCHW kernels, no pack
