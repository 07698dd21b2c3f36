// Micro-benchmark: the marching kernel's HBM access pattern for channel-group layouts of
// G = 4 (the shipped channel quads), 8, 16, 32 (NHWC) floats per pixel and group.
// One wave marches one band of rows of one 62-column strip (lanes = columns 62 s - 1 ..
// 62 s + 62); per row and channel group it loads the next f0 row of its column and the
// leading f1 tap pair (two horizontally adjacent pixels of the row below the warped
// position -- the tap cache of the real kernel supplies the other pair).  Every layout
// issues the same 16-byte loads per pixel row (C / 4 f0 + C / 2 f1); only the addresses
// differ.  80 KB of LDS per workgroup pins the real kernel's 2 workgroups per CU.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mbl tools/mb_layout.hip && /tmp/mbl
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                           \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

constexpr int W = 640, H = 480, C = 32, NP = 64, STRIPS = 11;
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ f32x4 bload(v4i, int, int, int) __asm("llvm.amdgcn.raw.buffer.load.v4f32");

__device__ inline v4i rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  v4i r;
  r.x = (int)(a & 0xffffffffu);
  r.y = (int)(a >> 32);
  r.z = (int)bytes;
  r.w = 0x00020000;
  return r;
}

// layout G: frame [C/G][H][W][G] floats; the 16-byte chunk k (0 .. C/4-1) of pixel (x, y)
// lies at ((k / (G/4)) * H * W + y * W + x) * G * 4 + (k % (G/4)) * 16 bytes
// MODE 0: the marching pattern; 1: f0 only; 2: f1 taps at the pixel's own column (no
// gather); 3: 64-column strips without halo columns (10 strips of 64); 4: grid split -- 3
// row bands x 11 strips = 33 segments with common row cuts (neighbouring strips march the
// same rows at the same time), wave w < 32 owns segment w, the 33rd is split 5 rows a wave
// and marched after it; 5: as 0 without the XCD-aware workgroup remap; 6: as 4 with a
// workgroup barrier every row (the 4 waves -- mostly 4 adjacent strips -- in lockstep);
// 7: as 4 plus the real kernel's two trailing tap loads per group, every lane re-requesting
// its leading pair (the tap cache's branch-free hit path: L1 hits); 8: as 4 plus the two
// trailing loads from one lane in eight only (EXEC-masked: the data path skips the hit lanes)
template <int G, int MODE = 0>
__global__ __launch_bounds__(256) void march(const float* f0, const float* f1, float* out, float rot, float shift) {
  __shared__ float pin[80 * 1024 / 4];  // the real kernel's LDS footprint: 2 workgroups per CU
  constexpr int NG = C / G, PER = G / 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // the shipped schedule at 64 pairs per launch: 8 workgroups (32 waves) per pair, each
  // wave a contiguous run of the pair's (strip, row) units in strip-major order
  constexpr int NS = MODE == 3 ? 10 : STRIPS, NW = 32, U = NS * H;
  // a pair's 8 workgroups on one XCD (the dispatcher deals workgroups round-robin over 8)
  const int kb = MODE == 5 ? blockIdx.x : (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  const int b = kb / 8, band = (kb % 8) * 4 + wave;
  const int ubeg = U * band / NW, uend = U * (band + 1) / NW;
  const uint32_t frame = (uint32_t)H * W * C * 4;
  const v4i r0 = rsrc(f0 + (size_t)b * H * W * C, frame), r1 = rsrc(f1 + (size_t)b * H * W * C, frame);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  constexpr bool GP = MODE == 4 || MODE == 6 || MODE == 7 || MODE == 8;
  const int nunits = GP ? 160 + 5 : uend - ubeg;
  for (int i = 0; i < nunits; ++i) {
    int s, y;
    if (MODE == 6) __syncthreads();
    if (GP) {
      const int seg = i < 160 ? band : 32, row = i < 160 ? i : 160 + 5 * band + (i - 160);
      s = seg % STRIPS;
      y = (seg / STRIPS) * 160 + (i < 160 ? row : row - 160);
    } else {
      s = (ubeg + i) / H;
      y = ubeg + i - s * H;
    }
    const int xs = MODE == 3 ? s * 64 + lane : s * 62 - 1 + lane, xc = min(max(xs, 0), W - 1);
    const int yn = min(y + 1, H - 1);
    const float fu = xc + rot * (y - H / 2) + shift, fv = y - rot * (xc - W / 2) + shift;
    const int tx = MODE == 2 ? min(xc, W - 2) : min(max((int)floorf(fu), 0), W - 2), ty = min(max((int)floorf(fv) + 1, 0), H - 1);
    // all 24 loads of the row in flight in every layout (equal memory-level parallelism);
    // a group's chunks are issued back to back (same cache lines)
    f32x4 l[5 * C / 4];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int gp = g * H * W;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        l[3 * (g * PER + k)] = bload(r0, ((gp + yn * W + xc) * G) * 4 + 16 * k, 0, 2);
        if (MODE != 1) {
          l[3 * (g * PER + k) + 1] = bload(r1, ((gp + ty * W + tx) * G) * 4 + 16 * k, 0, 0);
          l[3 * (g * PER + k) + 2] = bload(r1, ((gp + ty * W + tx + 1) * G) * 4 + 16 * k, 0, 0);
        } else {
          l[3 * (g * PER + k) + 1] = l[3 * (g * PER + k) + 2] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        f32x4& t0 = l[3 * C / 4 + 2 * (g * PER + k)];
        f32x4& t1 = l[3 * C / 4 + 2 * (g * PER + k) + 1];
        t0 = t1 = f32x4{0.f, 0.f, 0.f, 0.f};
        if (MODE == 7) {
          t0 = bload(r1, ((gp + ty * W + tx) * G) * 4 + 16 * k, 0, 0);
          t1 = bload(r1, ((gp + ty * W + tx + 1) * G) * 4 + 16 * k, 0, 0);
        } else if (MODE == 8 && (lane & 7) == 0) {
          const int tyt = max(ty - 1, 0);
          t0 = bload(r1, ((gp + tyt * W + tx) * G) * 4 + 16 * k, 0, 0);
          t1 = bload(r1, ((gp + tyt * W + tx + 1) * G) * 4 + 16 * k, 0, 0);
        }
      }
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int k = 0; k < 5 * C / 4; ++k) acc += l[k];
  }
  pin[threadIdx.x] = acc.x;
  if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[0] = pin[(threadIdx.x + 1) & 255];
}

template <int G, int MODE = 0>
void run(const float* f0, const float* f1, float* out) {
  const int grid = NP * 8;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) march<G, MODE><<<grid, 256>>>(f0, f1, out, 0.05f, 0.3f);
  CHECK(hipEventRecord(e0));
  const int reps = 20;
  for (int i = 0; i < reps; ++i) march<G, MODE><<<grid, 256>>>(f0, f1, out, 0.05f, 0.3f);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double alg = 2.0 * NP * H * W * C * 4;  // f0 + f1 once each
  static const char* modes[] = {"marching", "f0 only", "f1 at own column", "64-col strips", "grid 3x11 + pool",
                                "no XCD remap", "grid + row barrier", "grid + re-requests", "grid + 1/8 trailing"};
  printf("G=%2d %-17s: %7.1f us per launch, %6.0f GB/s algorithmic (f0 + f1)\n", G, modes[MODE], us,
         (MODE == 1 ? alg / 2 : alg) / (us * 1e-6) / 1e9);
}

int main(int argc, char** argv) {
  const int only = argc > 1 ? atoi(argv[1]) : -1;  // one G = 4 mode (for a PMC pass), or all
  const size_t n = (size_t)NP * C * W * H;
  float *f0, *f1, *out;
  CHECK(hipMalloc(&f0, n * 4));
  CHECK(hipMalloc(&f1, n * 4));
  CHECK(hipMalloc(&out, 4));
  CHECK(hipMemset(f0, 0, n * 4));
  CHECK(hipMemset(f1, 0, n * 4));
  if (only >= 0) {
    switch (only) {
      case 0: run<4, 0>(f0, f1, out); break;
      case 1: run<4, 1>(f0, f1, out); break;
      case 2: run<4, 2>(f0, f1, out); break;
      case 3: run<4, 3>(f0, f1, out); break;
      case 4: run<4, 4>(f0, f1, out); break;
      case 5: run<4, 5>(f0, f1, out); break;
      case 7: run<4, 7>(f0, f1, out); break;
      case 8: run<4, 8>(f0, f1, out); break;
      default: run<4, 6>(f0, f1, out); break;
    }
    return 0;
  }
  if (only == -2) {  // the tap-cache trailing-load question only
    for (int rep = 0; rep < 3; ++rep) {
      run<4, 4>(f0, f1, out);
      run<4, 7>(f0, f1, out);
      run<4, 8>(f0, f1, out);
    }
    return 0;
  }
  for (int rep = 0; rep < 2; ++rep) {
    run<4>(f0, f1, out);
    run<8>(f0, f1, out);
    run<16>(f0, f1, out);
    run<32>(f0, f1, out);
    run<4, 1>(f0, f1, out);
    run<4, 2>(f0, f1, out);
    run<4, 3>(f0, f1, out);
    run<4, 4>(f0, f1, out);
    run<4, 5>(f0, f1, out);
    run<4, 6>(f0, f1, out);
  }
  return 0;
}
