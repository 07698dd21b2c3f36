// Micro-benchmark of the reduce kernel's memory pattern alone (no Jacobian work):
// per pixel and channel, the f0 stencil rows and the 4 bilinear taps of f1 at a
// warped position.  Used to find the TA/TD cost of each access form.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mb tools/mb_gather.hip && /tmp/mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1);} } while (0)

constexpr int W = 640, H = 480, C = 32, B = 8;

typedef int v4i __attribute__((ext_vector_type(4)));
__device__ float __llvm_amdgcn_raw_buffer_load_f32(v4i, int, int, int) __asm("llvm.amdgcn.raw.buffer.load.f32");
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ f32x2 __llvm_amdgcn_raw_buffer_load_v2f32(v4i, int, int, int) __asm("llvm.amdgcn.raw.buffer.load.v2f32");

typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ f32x4 __llvm_amdgcn_raw_buffer_load_v4f32(v4i, int, int, int) __asm("llvm.amdgcn.raw.buffer.load.v4f32");

__device__ inline v4i rsrc(const void* p, uint32_t bytes) {
  uint64_t a = (uint64_t)p;
  v4i r;
  r.x = (int)(a & 0xffffffffu);
  r.y = (int)(a >> 32);
  r.z = (int)bytes;
  r.w = 0x00020000;
  return r;
}

// MODE bits: 1 = f0 rows (ROWS per pixel-row), 2 = f1 gathers (2 x dwordx2), 4 = f1 coalesced instead of gather,
// 8 = channel-blocked layout [B][C/4][H][W][4]: one dwordx4 per row / tap covers 4 channels,
// 16 = NHWC [B][H][W][C]: one dwordx4 per row / tap covers 4 channels of a 128-byte pixel record
template <int MODE, int R>
__global__ __launch_bounds__(256) void kern(const float* f0, const float* f1, float* out, float rot, float shift) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tiles_x = (W + 61) / 62, row_groups = (H + 4 * R - 1) / (4 * R);
  const int per_pair = tiles_x * row_groups;
  const int tile = blockIdx.x;
  const int b = tile / per_pair, local = tile % per_pair;
  const int ty = local / tiles_x, tx = local % tiles_x;
  const int y0 = ty * 4 * R + wave * R;
  const int xs = tx * 62 - 1 + lane;
  const int xc = min(max(xs, 0), W - 1);
  const uint32_t plane = W * H * 4;
  const v4i r0 = rsrc(f0 + (size_t)b * C * W * H, plane * C), r1 = rsrc(f1 + (size_t)b * C * W * H, plane * C);
  float acc = 0.f;
  int rows[R + 2];
  for (int j = 0; j < R + 2; ++j) rows[j] = min(max(y0 - 1 + j, 0), H - 1) * W * 4;
  int g0[R], g1[R];
  for (int r = 0; r < R; ++r) {
    const float y = (float)min(y0 + r, H - 1);
    const float u = xc + rot * (y - H / 2) + shift, v = y - rot * (xc - W / 2) + shift;
    const int x0 = min(max((int)floorf(u), 0), W - 2), yy = min(max((int)floorf(v), 0), H - 2);
    g0[r] = (yy * W + x0) * 4;
    g1[r] = g0[r] + W * 4;
  }
  if (MODE & 8) {
    f32x4 a4 = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < C; c += 4) {
      const int po = c * plane;  // = (c / 4) * (4 * plane): plane of a channel quad
      if (MODE & 1) {
        for (int j = 0; j < R + 2; ++j) a4 += __llvm_amdgcn_raw_buffer_load_v4f32(r0, (xc * 4 + rows[j]) * 4, po, 0);
      }
      if (MODE & 2) {
        for (int r = 0; r < R; ++r) {
          a4 += __llvm_amdgcn_raw_buffer_load_v4f32(r1, g0[r] * 4, po, 0);
          a4 += __llvm_amdgcn_raw_buffer_load_v4f32(r1, g0[r] * 4 + 16, po, 0);
          a4 += __llvm_amdgcn_raw_buffer_load_v4f32(r1, g1[r] * 4, po, 0);
          a4 += __llvm_amdgcn_raw_buffer_load_v4f32(r1, g1[r] * 4 + 16, po, 0);
        }
      }
    }
    acc = a4.x + a4.y + a4.z + a4.w;
  }
  if (MODE & 16) {
    f32x4 a4 = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < C; c += 4) {
      if (MODE & 1) {
        for (int j = 0; j < R + 2; ++j) a4 += __llvm_amdgcn_raw_buffer_load_v4f32(r0, (xc * 4 + rows[j]) * C, c * 4, 0);
      }
      if (MODE & 2) {
        for (int r = 0; r < R; ++r) {
          a4 += __llvm_amdgcn_raw_buffer_load_v4f32(r1, g0[r] * C, c * 4, 0);
          a4 += __llvm_amdgcn_raw_buffer_load_v4f32(r1, g0[r] * C + 4 * C, c * 4, 0);
          a4 += __llvm_amdgcn_raw_buffer_load_v4f32(r1, g1[r] * C, c * 4, 0);
          a4 += __llvm_amdgcn_raw_buffer_load_v4f32(r1, g1[r] * C + 4 * C, c * 4, 0);
        }
      }
    }
    acc = a4.x + a4.y + a4.z + a4.w;
  }
  for (int c = 0; c < ((MODE & 24) ? 0 : C); ++c) {
    const int po = c * plane;
    if (MODE & 1) {
      for (int j = 0; j < R + 2; ++j) acc += __llvm_amdgcn_raw_buffer_load_f32(r0, xc * 4 + rows[j], po, 0);
    }
    if (MODE & 2) {
      for (int r = 0; r < R; ++r) {
        if (MODE & 4) {
          acc += __llvm_amdgcn_raw_buffer_load_f32(r1, xc * 4 + rows[r + 1], po, 0);
          acc += __llvm_amdgcn_raw_buffer_load_f32(r1, xc * 4 + rows[r + 1] + W * 4, po, 0);
        } else {
          const f32x2 a = __llvm_amdgcn_raw_buffer_load_v2f32(r1, g0[r], po, 0);
          const f32x2 d = __llvm_amdgcn_raw_buffer_load_v2f32(r1, g1[r], po, 0);
          acc += a.x + a.y + d.x + d.y;
        }
      }
    }
  }
  if (acc == 12345.f) out[0] = acc;
}

template <int MODE, int R>
void run(const char* name, const float* f0, const float* f1, float* out, float rot, float shift) {
  const int tiles_x = (W + 61) / 62, row_groups = (H + 4 * R - 1) / (4 * R);
  const int grid = B * tiles_x * row_groups;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) kern<MODE, R><<<grid, 256>>>(f0, f1, out, rot, shift);
  CHECK(hipEventRecord(e0));
  const int reps = 20;
  for (int i = 0; i < reps; ++i) kern<MODE, R><<<grid, 256>>>(f0, f1, out, rot, shift);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-28s R=%d rot=%.3f: %7.1f us\n", name, R, rot, ms * 1e3 / reps);
}

int main() {
  const size_t n = (size_t)B * C * W * H;
  float *f0, *f1, *out;
  CHECK(hipMalloc(&f0, n * 4));
  CHECK(hipMalloc(&f1, n * 4));
  CHECK(hipMalloc(&out, 4));
  CHECK(hipMemset(f0, 0, n * 4));
  CHECK(hipMemset(f1, 0, n * 4));
  for (float rot : {0.05f}) {
    run<1, 1>("f0 rows", f0, f1, out, rot, 0.3f);
    run<1, 2>("f0 rows", f0, f1, out, rot, 0.3f);
    run<2, 1>("f1 gathers", f0, f1, out, rot, 0.3f);
    run<2, 2>("f1 gathers", f0, f1, out, rot, 0.3f);
    run<6, 1>("f1 coalesced", f0, f1, out, rot, 0.3f);
    run<3, 1>("f0 rows + f1 gathers", f0, f1, out, rot, 0.3f);
    run<3, 2>("f0 rows + f1 gathers", f0, f1, out, rot, 0.3f);
    run<7, 1>("f0 rows + f1 coalesced", f0, f1, out, rot, 0.3f);
    run<9, 1>("C4 f0 rows", f0, f1, out, rot, 0.3f);
    run<9, 2>("C4 f0 rows", f0, f1, out, rot, 0.3f);
    run<10, 1>("C4 f1 gathers", f0, f1, out, rot, 0.3f);
    run<11, 1>("C4 f0 rows + f1 gathers", f0, f1, out, rot, 0.3f);
    run<11, 2>("C4 f0 rows + f1 gathers", f0, f1, out, rot, 0.3f);
    run<17, 1>("NHWC f0 rows", f0, f1, out, rot, 0.3f);
    run<18, 1>("NHWC f1 gathers", f0, f1, out, rot, 0.3f);
    run<19, 1>("NHWC f0 rows + f1 gathers", f0, f1, out, rot, 0.3f);
    run<19, 2>("NHWC f0 rows + f1 gathers", f0, f1, out, rot, 0.3f);
  }
  return 0;
}
