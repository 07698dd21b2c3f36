"""Read bandwidth vs working-set size (dpft_read_probe): HBM streaming vs Infinity-Cache (MALL)
hits.  python tools/mall_probe.py"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from deep_prob_feature_track_amd import _native as N, ic  # noqa: E402

dev = torch.device("cuda:0")
L = N.lib()
out = torch.empty(int(L.dpft_read_probe_out_floats()), dtype=torch.float32, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
for mb in (16, 32, 64, 128, 192, 256, 512, 2048, 10240):
    n = mb << 20
    buf = torch.ones(n // 4, dtype=torch.float32, device=dev)
    for nt in (0, 1):
        run = lambda: N.check(L.dpft_read_probe(ic._ptr(buf), n, nt, ic._ptr(out), st), "read probe")
        for _ in range(5):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = max(3, min(200, (40 << 30) // n))
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        s = e0.elapsed_time(e1) * 1e-3 / reps
        print(f"{mb:6d} MB nt={nt}: {n / s / 1e12:.2f} TB/s", flush=True)
    del buf
