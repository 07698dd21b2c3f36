"""Write tools/_var/sync.hip: the shipped kernel source with a soft row-step sync among the four
waves of a marching workgroup (A/B experiment).

Each wave publishes its row-step index in LDS; before a step it waits (s_sleep) while it is
more than DPFT_SYNC_SLACK steps ahead of the slowest wave of its workgroup (bounded spin; the
slowest wave never waits, so there is no deadlock).  Build with
    python tools/build_variants.py s2=@tools/_var/sync.hip:-DDPFT_SYNC_SLACK=2
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "deep_prob_feature_track_amd", "csrc", "dpft_ic.hip")).read()

a = "  __shared__ f32x4 lds_win[kWin ? 4 : 1][kWin ? 2 * (CT / 4) * 64 : 1];  // used: 2 x NQW quads per wave\n"
assert a in src
src = src.replace(a, a + "  __shared__ int lds_prog[4];\n")

b = "    for (int k = 0; k < nrows; ++k) step(k);\n"
assert b in src
sync = r"""    if (lane == 0) lds_prog[wave] = 0;
    __syncthreads();
    for (int k = 0; k < nrows; ++k) {
      if ((k & (DPFT_SYNC_EVERY - 1)) == 0) {
        __hip_atomic_store(&lds_prog[wave], k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        for (int spin = 0; spin < 4096; ++spin) {
          const int v = __hip_atomic_load(&lds_prog[lane & 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const int m = min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 1)),
                            min(__builtin_amdgcn_readlane(v, 2), __builtin_amdgcn_readlane(v, 3)));
          if (k - m <= DPFT_SYNC_SLACK) break;
          __builtin_amdgcn_s_sleep(1);
        }
      }
      step(k);
    }
    __hip_atomic_store(&lds_prog[wave], 1 << 30, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
"""
src = src.replace(b, sync)
src = "#ifndef DPFT_SYNC_SLACK\n#define DPFT_SYNC_SLACK 2\n#endif\n#ifndef DPFT_SYNC_EVERY\n#define DPFT_SYNC_EVERY 1\n#endif\n" + src
os.makedirs(os.path.join(ROOT, "tools", "_var"), exist_ok=True)
open(os.path.join(ROOT, "tools", "_var", "sync.hip"), "w").write(src)
print("tools/_var/sync.hip")
