// libdpft_ic.so -- gfx950 (MI355X) kernels + C ABI for the trust-region
// inverse-compositional (U_IC) solver of Deep Probabilistic Feature-metric
// Tracking.  ABI and semantics: include/dpft_ic.h.
//
// One Gauss-Newton iteration at one pyramid level is ONE launch:
//
//   ic_reduce_kernel   fused, HBM-bound pass over every pixel of every pair:
//                      inverse-depth warp (geometry.py:291-323), bilinear
//                      gathers of invD1 / f1 / sigma1 (geometry.py:353-365),
//                      occlusion + object masks (geometry.py:334-350,
//                      algorithms.py:1999-2008), uncertainty-weighted residual
//                      (algorithms.py:1960-1989), Sobel gradients of f0 and
//                      sigma0 recomputed in registers with DPP lane shifts
//                      (algorithms.py:1844-1865, never stored), the per-channel
//                      inverse Jacobian (algorithms.py:867-887, 1867-1917)
//                      folded into channel sums, and the 21 + 6 normal-equation
//                      partials (algorithms.py:812-834).  Each workgroup writes
//                      one fixed-size record: no atomics on data, deterministic.
//                      The LAST workgroup to finish (threadfence handshake) then
//                      reduces every pair's records in a fixed order in fp64,
//                      applies the batch-global truncated-sigma correction,
//                      Levenberg damping, the 6x6 solve and the SE(3) update
//                      (algorithms.py:2017-2103), in place.
//
// plus, on the first iteration of a level, minmax_kernel (sigma0 extrema).
//
// J is never materialised: per pixel and channel the reference's J_c is
// -(a_c Jx + b_c Jy), so sum_c J_c J_c^T = Saa JxJx^T + Sab (JxJy^T + JyJx^T)
// + Sbb JyJy^T and sum_c J_c rw_c = -(Sar Jx + Sbr Jy): channel sums per pixel
// replace the [B,C,HW,6] tensor of algorithms.py:878-885.
//
// Truncated sigma (algorithms.py:1975-1980) compares sigma_r against its min /
// max over the WHOLE batch, which is only known after the pass.  Because J is
// unmasked the flag only changes JtR, so each record also carries the block's
// sigma_r extrema and the JtR correction sum_c J_c (1e-6 - rw_c) of the
// not-yet-invalid pixels that attain them; the finalize applies the
// corrections of the blocks whose extremum equals the global one.
//
// The equality tests of that mask (and u > 0 of the in-view test) make the
// result depend on the last bit of the warped coordinates, so the warp and the
// sampler reproduce the reference's CPU arithmetic op for op (measured, see
// warp_point / bil4); everywhere else the compiler may contract freely.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "dpft_ic.h"
#include "dpft_tuning.h"

// LLVM buffer-load intrinsics (declared at global scope: they bind by asm label).
typedef int Rsrc __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ float llvm_buf_load_f32(Rsrc r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.f32");
__device__ f32x2 llvm_buf_load_f32x2(Rsrc r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.v2f32");
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ f32x4 llvm_buf_load_f32x4(Rsrc r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");

namespace {

constexpr int kThreads = 256;          // 4 waves of 64
constexpr int kTileW = 64;             // one wave = 64 consecutive pixels of a row
constexpr int kRowsPerStep = 4;        // one row per wave per step
constexpr int kRing = 2;               // tile paths: load slots in flight (kRing - 1 units ahead)
constexpr int kCK = 2;                 // tile paths, NCHW: channels per pipeline unit
constexpr int kRPL = 1;                // image rows per lane (one sigma plane, NCHW)
constexpr int kRPL4 = 1;               // image rows per lane (channel-quad tile path)
constexpr int kMaxSteps = 4;           // tile paths: up to 4 * kMaxSteps rows per workgroup
// channel-quad levels of at most kSplitMaxPixels per pair (and kSplitMaxLaunchPixels per
// launch, all pairs): ic_split_kernel; larger ones march (a level of a grouped call with
// more -- level 2 of 32 pairs: 614 k pixels, the size of level 1 of 8 pairs -- fills the
// device as a marching launch)
constexpr long kSplitMaxPixels = DPFT_SPLIT_MAX_PIXELS;
constexpr long kSplitMaxLaunchPixels = DPFT_SPLIT_MAX_LAUNCH_PIXELS;
constexpr int kMarchSkew = DPFT_MARCH_SKEW;  // band-size skew of the marching schedule (64ths, 0..63)
constexpr int kMarchMinRows = DPFT_MARCH_MIN_ROWS;  // marching: minimum rows per wave (0: none)
constexpr int kRingQ = DPFT_RING_Q;          // marching quad loop: quads in flight (kRingQ - 1 ahead)
constexpr int kF0Aux = 2;                    // cache policy of the marching f0 stream (nt: used once)
constexpr int kGridWaste = DPFT_GRID_WASTE;  // marching band grid: idle waves allowed (64ths of a pair's)

// ---- reduce-record layout (floats) ------------------------------------------
constexpr int kRec = 48;
constexpr int kIcpRec = 32;  // icp_records_kernel record: JtJ (21) + JtR (6) + 0 (the invalid count's slot), padded
constexpr int kIcpSub = DPFT_ICP_SUB;  // icp_records_kernel: at most this many workgroups (records) per reduce slot
constexpr int kIcpTab = 2048;  // icp_records_kernel: normalised-coordinate table in LDS when W + H fits
constexpr int R_NINV = 27;    // invalid pixels (occlusion | masks | sigma0-trunc)
constexpr int R_MN_ALL = 28;  // min of sigma_r over every channel
constexpr int R_MN0 = 29;     // min of sigma_r channel 0
constexpr int R_CMN = 30;     // 6: JtR correction of the pixels at R_MN0
constexpr int R_NMN = 36;     // count of those pixels
constexpr int R_MX_ALL = 37;
constexpr int R_MX0 = 38;
constexpr int R_CMX = 39;     // 6
constexpr int R_NMX = 45;

// ---- residual-record layout --------------------------------------------------
constexpr int L_SUM = 0, L_NINV = 1, L_MN_ALL = 2, L_MN0 = 3, L_LMN = 4, L_NMN = 5,
              L_MX_ALL = 6, L_MX0 = 7, L_LMX = 8, L_NMX = 9;

// workspace: [ctrl 8 KiB][records].  ctrl words: sigma0 extrema (order-encoded),
// the two "blocks done" counters of the last-block finalizers, and the per-block
// partial extrema of the sigma0 pass.  The counters are zero between calls: the
// caller zero-fills the workspace once, every last block resets its counter.
// kCtlMMDoneL / kCtlExtSlots: dpft_sigma_extrema_levels' per-level completion counters and
// the per-level sigma0 extrema it leaves (DPFT_EXT_SLOT / DPFT_EXTREMA_READY)
constexpr int kCtlMMDoneL = 10, kCtlExtSlots = 16, kMaxExtSlots = 8;
constexpr int kCtlMin = 0, kCtlMax = 1, kCtlDone = 2, kCtlMMDone = 3, kCtlD1Min = 8,
              kCtlPart = 64, kCtlPair = 1152;
constexpr int kMaxMMBlocks = 512;
// pair_reduce2's LDS scratch: 42 fields x 65 quad rows (the extrema exchange overlaps it)
constexpr int kFinScratch = 42 * 65;
// cache-policy operand of the raw buffer intrinsics: sc1 (agent-coherent; gfx940+ bit 4)
constexpr int kAuxSc1 = 16;
// minmax_kernel: workgroups (<= kMaxMMBlocks) and 16-byte loads in flight per thread.
// Its last-workgroup reduction serialises one counter arrival per workgroup.
constexpr int kMMGrid = DPFT_MM_GRID, kMMLoads = DPFT_MM_LOADS;
static_assert(kMMGrid <= kMaxMMBlocks, "minmax partials");
static_assert(kMarchSkew >= 0 && kMarchSkew < 64, "band skew in 64ths");
constexpr int kMaxPairs = 2048;  // per call (one completion counter per pair)
constexpr int kMaxGrid = 4096;   // reduce-kernel workgroups (resident capacity is far below)
// Independent batches in one call (DPFT_GROUP): per batch a completion counter of the
// batch solve (kCtlGDone + g), sigma0 extrema per (slot, batch) (kCtlGExt; slot index
// kMaxExtSlots = a call without DPFT_EXT_SLOT) and the pre-pass counters per (level, batch).
constexpr int kMaxGroups = 32;
constexpr int kCtlGDone = 32, kCtlGExt = 4096, kCtlGMMDone = kCtlGExt + 2 * (kMaxExtSlots + 1) * kMaxGroups;
// combine_ICP: depth1 extrema per independent batch (the normal map's invalid-depth test)
constexpr int kCtlGD1 = kCtlGMMDone + 4 * kMaxGroups;
constexpr size_t kCtrlBytes = 20480;
static_assert((kCtlGD1 + 2 * kMaxGroups) * 4 <= kCtrlBytes, "ctrl area (batch depth extrema)");
static_assert(kCtlGDone + kMaxGroups <= kCtlPart, "batch counters");
static_assert((kCtlGMMDone + 4 * kMaxGroups) * 4 <= kCtrlBytes, "ctrl area (batches)");
static_assert((kCtlPart + 2 * kMaxMMBlocks) * 4 <= kCtlPair * 4, "ctrl area");
static_assert((kCtlPair + kMaxPairs) * 4 <= kCtrlBytes, "ctrl area");
// per-pair record (fp64) written by the last workgroup of each pair
constexpr int P_S = 0;        // 28: JtJ upper (21), JtR (6), #invalid
constexpr int P_CMN = 28;     // 7: JtR / count corrections of the blocks at the pair's min sigma_r ch0
constexpr int P_CMX = 35;     // 7: same at the max
constexpr int P_MN_ALL = 42, P_MN0 = 43, P_MX_ALL = 44, P_MX0 = 45;
constexpr int kPRec = 48;

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

// ------------------------------------------------------------------ device utils
__device__ __forceinline__ uint32_t enc_ord(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float dec_ord(uint32_t e) {
  uint32_t u = (e & 0x80000000u) ? (e & 0x7fffffffu) : ~e;
  return __uint_as_float(u);
}

// Threadfence-reduction handshake: every workgroup publishes its record, then
// the one that arrives last (counter == total-1) sees all records and finalizes.
// Agent-scope fences make the records of workgroups on other XCDs visible.
// Records cross workgroups (and XCDs, whose L2s are not coherent with each
// other) only through agent-scope relaxed atomic stores / loads (sc1: coherent
// at the device level), so the handshake needs no agent-scope fence -- whose
// L2 write-back / invalidate per workgroup would wreck the streaming reuse.
// Each wave waits for its record stores to be acknowledged before the barrier;
// only then does thread 0 bump the counter.
template <class T>
__device__ __forceinline__ void st_ag(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T ld_ag(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ bool block_is_last(uint32_t* counter, uint32_t add, uint32_t total) {
  __shared__ int s_last;
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's stores are complete
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(counter, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev + add == total;
    if (last) st_ag(counter, 0u);  // ready for the next launch
    s_last = last;
  }
  __syncthreads();
  return s_last != 0;
}

template <int W_>
struct WaveIdx {  // compile-time index tag (wave, row, buffer parity)
  static constexpr int value = W_;
};

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// XCD-aware bijective remap: the dispatcher deals workgroups round-robin over the
// 8 XCDs, so give the workgroups that share an XCD consecutive tiles (vertically
// adjacent tiles share halo rows through that XCD's L2).  Speed only.
__device__ __forceinline__ int xcd_remap(int orig, int n) {
  const int xcd = orig & 7, q = n >> 3, r = n & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

// ic_reduce_kernel: blockIdx -> (pair-major) workgroup slot.  xcd_remap keeps a pair's
// workgroups on one XCD; with several pairs per XCD (B > 8 at the resident grid) the
// workgroups of each pair are also taken half from the XCD's first dispatch round (the
// first workgroup on each CU, favoured by the oldest-first issue arbitration) and half
// from the second, as with one pair per XCD -- the band skew assumes exactly that split.
// Without it the second pair of an XCD ran entirely as second workgroups and finished
// last (B = 16: 313 us per level-0 launch, 156 us per 8 pairs against 141 at B = 8).
// `qr`: workgroups per XCD and dispatch round (the resident grid / 8; a grid of several
// rounds runs the pairs of round k of every XCD after those of round k - 1).
__device__ __forceinline__ int pair_slot_remap(int orig, int n, int nbpp, int qr) {
  int kb = xcd_remap(orig, n);
  const int q = n >> 3;
  if ((n & 7) == 0 && qr > 0 && q % qr == 0) {
    const int xb = kb - kb % q, i0 = kb - xb, rb = i0 - i0 % qr, i = i0 - rb;
    if ((nbpp & 1) == 0 && qr % nbpp == 0 && qr / nbpp >= 2 && (qr & 1) == 0) {
      const int h = qr >> 1, hp = nbpp >> 1;
      const bool second = i >= h;
      const int ii = second ? i - h : i, pin = ii / hp;
      kb = xb + rb + pin * nbpp + (ii - pin * hp) + (second ? hp : 0);
    }
  }
  return kb;
}

struct Taps {
  int o00, o01, o10, o11;
  int ob0, ob1;  // pair bases (row y0 / y1, column min(x0, W-2))
  bool lo;       // x0 < W-1: the pair's first element is the (x0) tap
  float nw, ne, sw, se;
};

// geometry.py:359-364 normalises u,v to [-1,1]; grid_sample(align_corners=True,
// padding_mode='border') maps back with (g + 1) * (size - 1) / 2, clamps to
// [0, size-1], and weighs the four neighbours by products of the distances.
// a / b for a divisor b that is constant across the launch, given rb = RN(1 / b): one product
// and one FMA correction (Markstein's theorem: with rb the correctly rounded reciprocal and the
// product within an ulp of the quotient, q + (a - b q) rb rounds to the correctly rounded
// quotient).  make_taps_xy uses it on |a| <= 2^30 (larger and NaN coordinates are clamped
// there first: the taps clamp to the image border either way), where only quotients of
// magnitude >= 2^-25 can move a tap; in that domain it equals the IEEE division for every
// float a: tools/div_check.c checks all 2^32 floats for b = 319.5, 159.5, 79.5, 39.5, 19.5, 9.5,
// 239.5, 119.5, 59.5, 29.5, 14.5, 7 (every level of 640x480 and 160x120) and a stride through
// all floats for every b = (n - 1) / 2, n = 2 .. 8192; the library selects it only for those
// twelve sizes (kVerifiedTapSizes), any other size divides by IEEE.
__device__ __forceinline__ float div_const(float a, float b, float rb) {
  const float q = a * rb;
  return __builtin_fmaf(__builtin_fmaf(-q, b, a), rb, q);
}
// RC: rs = RN(1 / sx), RN(1 / sy) given (the combine_ICP pass computes them once per workgroup)
template <bool RC = false>
__device__ __forceinline__ Taps make_taps_xy(float u, float v, int H, int W, int& tx0, int& tx1, int& ty0,
                                             int& ty1, const float* rs = nullptr) {
#pragma clang fp contract(off)
  const float sx = (float)(W - 1) * 0.5f;
  const float sy = (float)(H - 1) * 0.5f;
  float ix, iy;
  if constexpr (RC) {
    const float uc = fminf(fmaxf(u, -0x1p30f), 0x1p30f), vc = fminf(fmaxf(v, -0x1p30f), 0x1p30f);
    ix = (div_const(uc, sx, rs[0]) - 1.0f + 1.0f) * sx;
    iy = (div_const(vc, sy, rs[1]) - 1.0f + 1.0f) * sy;
  } else {
    ix = ((u / sx) - 1.0f + 1.0f) * sx;
    iy = ((v / sy) - 1.0f + 1.0f) * sy;
  }
  ix = fminf(fmaxf(ix, 0.0f), (float)(W - 1));
  iy = fminf(fmaxf(iy, 0.0f), (float)(H - 1));
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const int x0 = (int)fx0, y0 = (int)fy0;
  const float w = ix - fx0, e = 1.0f - w;
  const float n = iy - fy0, s = 1.0f - n;
  const int x1 = min(x0 + 1, W - 1), y1 = min(y0 + 1, H - 1);
  Taps t;
  t.o00 = y0 * W + x0;
  t.o01 = y0 * W + x1;
  t.o10 = y1 * W + x0;
  t.o11 = y1 * W + x1;
  const int xb = min(x0, W - 2);
  t.ob0 = y0 * W + xb;
  t.ob1 = y1 * W + xb;
  t.lo = x0 == xb;
  t.nw = s * e;
  t.ne = s * w;
  t.sw = n * e;
  t.se = n * w;
  tx0 = x0;
  tx1 = x1;
  ty0 = y0;
  ty1 = y1;
  return t;
}
__device__ __forceinline__ Taps make_taps(float u, float v, int H, int W) {
  int a, b, c, d;
  return make_taps_xy(u, v, H, W, a, b, c, d);
}

// An out-of-range neighbour always has weight exactly 0 under border clamping,
// so reading the clamped pixel instead of a masked zero changes nothing.  The
// accumulation is the fused chain the CPU grid sampler compiles to,
// fma(d, se, fma(c, sw, fma(b, ne, a * nw))): measured bit-identical to
// torch.nn.functional.grid_sample on 2e5 random samples.
__device__ __forceinline__ float bil4(float a, float b, float c, float d, const Taps& t) {
#pragma clang fp contract(off)
  return __builtin_fmaf(d, t.se, __builtin_fmaf(c, t.sw, __builtin_fmaf(b, t.ne, a * t.nw)));
}
__device__ __forceinline__ float bil(const float* __restrict__ p, const Taps& t) {
  return bil4(p[t.o00], p[t.o01], p[t.o10], p[t.o11], t);
}
// Channel c of a feature tensor in NCHW (stride 1) or channel-quad layout (stride 4).
__device__ __forceinline__ const float* chan_base(const float* fb, int c, int HW, bool c4) {
  return c4 ? fb + (size_t)(c >> 2) * 4 * HW + (c & 3) : fb + (size_t)c * HW;
}
__device__ __forceinline__ float bil_s(const float* __restrict__ p, const Taps& t, int s) {
  return bil4(p[t.o00 * s], p[t.o01 * s], p[t.o10 * s], p[t.o11 * s], t);
}
__device__ __forceinline__ float bil_u8(const uint8_t* __restrict__ p, const Taps& t) {
  return bil4((float)p[t.o00], (float)p[t.o01], (float)p[t.o10], (float)p[t.o11], t);
}

struct Warp {
  float u, v, iz, xr, yr;
};

// Inverse-depth warp of pixel (x, y), op for op as the reference evaluates it on
// the CPU (geometry.py:63-85, 291-323): px = (u - cx) / fx; torch.bmm(R, [px,py,1])
// = fma(R1, py, R0 * px) + R2 per row (measured bit-identical for every
// shape used); + t * invD; u = (X / Z) * fx + cx; iz = invD / Z.
// the normalised pixel coordinates px = (u - cx) / fx, py = (v - cy) / fy
__device__ __forceinline__ float norm_coord(int x, float c, float f) {
#pragma clang fp contract(off)
  return ((float)x - c) / f;
}
__device__ __forceinline__ Warp warp_point_n(float xr, float yr, float d, const float* __restrict__ Rm,
                                             const float* __restrict__ tv, float fx, float fy, float cx, float cy) {
#pragma clang fp contract(off)
  Warp w;
  w.xr = xr;
  w.yr = yr;
  const float X = (__builtin_fmaf(Rm[1], w.yr, Rm[0] * w.xr) + Rm[2]) + tv[0] * d;
  const float Y = (__builtin_fmaf(Rm[4], w.yr, Rm[3] * w.xr) + Rm[5]) + tv[1] * d;
  const float Z = (__builtin_fmaf(Rm[7], w.yr, Rm[6] * w.xr) + Rm[8]) + tv[2] * d;
  w.u = (X / Z) * fx + cx;
  w.v = (Y / Z) * fy + cy;
  w.iz = d / Z;
  return w;
}
__device__ __forceinline__ Warp warp_point(int x, int y, float d, const float* __restrict__ Rm,
                                           const float* __restrict__ tv, float fx, float fy, float cx, float cy) {
  return warp_point_n(norm_coord(x, cx, fx), norm_coord(y, cy, fy), d, Rm, tv, fx, fy, cx, cy);
}

// Last-block finalize parameters (one record per workgroup, fixed-order fp64 sums).
struct FinParams {
  const float* rec;
  const float* icp_rec;  // combine_ICP on the channel-quad path: [B][nbpp][icp_sub][kIcpRec] records of
                         // icp_records_kernel (JtJ 21 + JtR 6), added to the reduce records; null: none
  int icp_sub;           // icp_records_kernel workgroups per reduce workgroup slot (1 .. kIcpSub)
  int nbpp, B;        // reduce kernel: workgroups (records) per pair, pairs
  double* prec;       // [B][kPRec] per-pair records
  uint32_t* pair_cnt; // [B] completion counters
  uint32_t* done_cnt; // pairs finished (one counter per independent batch)
  int group;          // pairs per independent batch (B: the call is one batch)
  int nblocks, per_pair, HW;
  uint32_t flags;
  int no_update;      // DPFT_ITER_NO_UPDATE: normal equations out, pose unchanged
  float* R;
  float* t;
  float* jtj_out;
  float* jtr_out;
  int32_t* invalid_out;
  float* loss_out;
  uint32_t* status;
};

struct IterParams {
  const float* f0;
  const float* f1;
  const float* s0;
  const float* s1;
  const float* invD0;
  const float* invD1;
  const uint8_t* mask0;
  const uint8_t* mask1;
  const float* wgt;      // NO_UNCERTAINTY: per-pixel M-estimator weights [B,1,H,W] (nullable)
  const float* depth0;   // COMBINE_ICP: raw depth pyramids level (max-pooled), [B,1,H,W]
  const float* depth1;
  const f32x4* nrm1;     // COMBINE_ICP: frame 1's [nx, ny, nz, depth1] map, [B,H,W] (workspace, per level)
  float* icp_rec;        // COMBINE_ICP: icp_records_kernel's records (workspace)
  float icp_w;           // ScaleNet('None') weight (algorithms.py:1563)
  const float* K;
  const float* R;
  const float* t;
  int B, C, Cs, H, W;
  int tiles_x, tiles_y, steps, nblocks;
  uint32_t flags;
  uint32_t* ctrl;        // see kCtl*
  const uint32_t* ext;   // sigma0 extrema of this level (order-encoded min, max)
  float* rec;
  int nbpp, per_pair, row_groups, rps;  // reduce kernel schedule (see ic_reduce_kernel); rps = rows per step
  int round_wg;    // reduce kernel: resident workgroups per XCD (pair_slot_remap)
  int fin_on;      // 0: records only (timing hook); 1: last workgroup finalizes
  int reverse;     // marching path: walk every band in the opposite direction (DPFT_ITER_REVERSE)
  int skew;        // marching path: band-size skew, 64ths (see ic_reduce_kernel)
  int rc_taps;     // combine_ICP pass: the taps' divisions by div_const (W and H verified sizes)
  FinParams fin;
};

// Per-pixel state that lives across the channel loop of one step.
struct PixelFrame {
  Taps tp;
  float d, xr, yr;
  float inv_s, kk, hx, hy, sr0, srmin, srmax;
  bool invalid;
};

// Warp, taps, occlusion (geometry.py:334-350) and object masks (algorithms.py:1999-2008).
__device__ __forceinline__ void setup_pixel(const IterParams& p, int b, int x, int y, float d,
                                            const float* __restrict__ Rm, const float* __restrict__ tv, float fx,
                                            float fy, float cx, float cy, PixelFrame& px) {
  const int W = p.W, H = p.H, HW = H * W;
  const Warp w = warp_point(x, y, d, Rm, tv, fx, fy, cx, cy);
  px.tp = make_taps(w.u, w.v, H, W);
  px.d = d;
  px.xr = w.xr;
  px.yr = w.yr;
  const float d1w = bil(p.invD1 + (size_t)b * HW, px.tp);
  const bool ok = (w.iz > d1w - 0.1f) && (w.u > 0.0f) && (w.u < (float)W) && (w.v > 0.0f) && (w.v < (float)H);
  bool inv = !ok;
  if (p.mask0) inv = inv || (p.mask0[(size_t)b * HW + y * W + x] == 0);
  if (p.mask1) inv = inv || !(bil_u8(p.mask1 + (size_t)b * HW, px.tp) > 0.0f);
  px.invalid = inv;
}

// Warp Jacobian at the origin, xi = [rot, trs] (algorithms.py:1908-1917).
__device__ __forceinline__ void warp_jac(float xr, float yr, float d, float fx, float fy, float* Jx, float* Jy) {
  const float xy = xr * yr;
  Jx[0] = -xy * fx;
  Jx[1] = (1.0f + xr * xr) * fx;
  Jx[2] = -yr * fx;
  Jx[3] = d * fx;
  Jx[4] = 0.0f;
  Jx[5] = -d * xr * fx;
  Jy[0] = (-1.0f - yr * yr) * fy;
  Jy[1] = xy * fy;
  Jy[2] = xr * fy;
  Jy[3] = 0.0f;
  Jy[4] = d * fy;
  Jy[5] = -d * yr * fy;
}

struct Extremum {
  float all;   // extremum over every channel (decides the global value)
  float v0;    // extremum of channel 0 (decides which pixels are flagged)
  float c[6];  // JtR correction of the not-yet-invalid pixels at v0
  float n;     // their count
};

template <bool IS_MIN>
__device__ __forceinline__ void ext_merge(Extremum& e, float all, float v0, const float* c, float n) {
  e.all = IS_MIN ? fminf(e.all, all) : fmaxf(e.all, all);
  const bool better = IS_MIN ? (v0 < e.v0) : (v0 > e.v0);
  if (better) {
    e.v0 = v0;
#pragma unroll
    for (int k = 0; k < 6; ++k) e.c[k] = c[k];
    e.n = n;
  } else if (v0 == e.v0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) e.c[k] += c[k];
    e.n += n;
  }
}

template <bool IS_MIN>
__device__ __forceinline__ void ext_wave_reduce(Extremum& e) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    Extremum o;
    o.all = __shfl_xor(e.all, off);
    o.v0 = __shfl_xor(e.v0, off);
#pragma unroll
    for (int k = 0; k < 6; ++k) o.c[k] = __shfl_xor(e.c[k], off);
    o.n = __shfl_xor(e.n, off);
    ext_merge<IS_MIN>(e, o.all, o.v0, o.c, o.n);
  }
}

// ---------------------------------------------------------------- buffer loads
// Raw buffer loads: a scalar resource per tensor plane-set, a per-lane byte
// offset that is fixed per pixel (or per tile column) and a scalar offset per
// channel / row -- no vector ALU spent on addresses, and an offset past the
// plane set reads 0 instead of faulting.  (The LLVM intrinsics are used
// directly: ROCm 7.2's __builtin_amdgcn_raw_buffer_load_b64 drops the second
// dword on gfx950.)

__device__ __forceinline__ Rsrc rsrc(const void* p, uint32_t bytes) {
  const unsigned long long a = (unsigned long long)p;
  Rsrc r;
  r.x = (int)(uint32_t)a;
  r.y = (int)(uint32_t)(a >> 32);  // stride 0
  r.z = (int)bytes;
  r.w = 0x00020000;
  return r;
}
__device__ __forceinline__ float bld(Rsrc r, int voff, int soff) { return llvm_buf_load_f32(r, voff, soff, 0); }
__device__ __forceinline__ f32x2 bld2(Rsrc r, int voff, int soff) { return llvm_buf_load_f32x2(r, voff, soff, 0); }
__device__ __forceinline__ f32x4 bld4(Rsrc r, int voff, int soff) { return llvm_buf_load_f32x4(r, voff, soff, 0); }

struct Gather4 {
  float a, b, c, d;  // the two loaded pairs: (row y0: a, b), (row y1: c, d)
};
// The two taps of a sampling row are adjacent columns: one 8-byte load each.
// The pair starts at min(x0, W-2) so it never leaves the row.  At x0 = W-1 the
// clamped neighbour x1 = x0 is the pair's SECOND element and its weights ne, se
// are exactly 0 (border clamp: ix = W-1 = x0); PairWeights moves nw, sw onto the
// second element instead of selecting values per channel:
// fma(p1y, sw, fma(p1x, 0, fma(p0y, nw, p0x * 0))) equals the reference's
// fma(d, 0, fma(c, sw, fma(b, 0, a * nw))) bit for bit (finite inputs).
__device__ __forceinline__ Gather4 gather4(Rsrc r, const Taps& t, int soff) {
  const f32x2 p0 = bld2(r, t.ob0 * 4, soff);
  const f32x2 p1 = bld2(r, t.ob1 * 4, soff);
  Gather4 g;
  g.a = p0.x;
  g.b = p0.y;
  g.c = p1.x;
  g.d = p1.y;
  return g;
}
struct PairWeights {
  float w0, w1, w2, w3;
};
__device__ __forceinline__ PairWeights pair_weights(const Taps& t) {
  PairWeights w;
  w.w0 = t.lo ? t.nw : 0.0f;
  w.w1 = t.lo ? t.ne : t.nw;
  w.w2 = t.lo ? t.sw : 0.0f;
  w.w3 = t.lo ? t.se : t.sw;
  return w;
}
__device__ __forceinline__ float bilp(const Gather4& g, const PairWeights& w) {
#pragma clang fp contract(off)
  return __builtin_fmaf(g.d, w.w3, __builtin_fmaf(g.c, w.w2, __builtin_fmaf(g.b, w.w1, g.a * w.w0)));
}

// ---------------------------------------------------------------- stencil by DPP
// No LDS and no workgroup barrier on the hot loop.  A wave owns one image row per
// step; lane l holds image column x0 - 1 + l (clamped = replicate padding), so a
// tile is 62 output pixels wide and lanes 0 and 63 only carry the halo.  Per
// channel every lane loads its own column in rows y-1, y, y+1 (three coalesced
// 256-byte loads) and forms the separable Sobel: V = top + 2 mid + bottom,
// D = bottom - top, gx = V(l+1) - V(l-1), gy = D(l-1) + 2 D(l) + D(l+1), the
// neighbour columns coming from DPP wave_shr:1 / wave_shl:1 lane shifts.
constexpr int kTileOut = kTileW - 2;  // output pixels per tile row

__device__ __forceinline__ float lane_from_left(float v) {  // lane l gets lane l - 1
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float lane_from_right(float v) {  // lane l gets lane l + 1
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, true));
}

// Unit-normalised Sobel from the three rows of this lane's column (algorithms.py:1852-1863).
// c ? a : b for a wave-uniform c, always as one v_cndmask: a select whose operand is a
// load can otherwise become a branch, and the copies on its two paths wait for every load
// in flight (the waitcnt pass cannot tell which path issued what)
__device__ __forceinline__ float sel_uniform(bool c, float a, float b) {
  float r;
  const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane(c ? -1 : 0);  // in SGPRs
  asm("v_cndmask_b32 %0, %2, %1, %3" : "=v"(r) : "v"(a), "v"(b), "s"(((uint64_t)m << 32) | m));
  return r;
}

__device__ __forceinline__ void sobel_cols(float top, float mid, float bot, float& gx, float& gy) {
  const float V = top + 2.0f * mid + bot;
  const float D = bot - top;
  const float x = lane_from_right(V) - lane_from_left(V);
  const float y = (lane_from_left(D) + 2.0f * D) + lane_from_right(D);
  const float inv = __builtin_amdgcn_rsqf(x * x + y * y + 1e-8f);  // argument >= 1e-8: no denormal path
  gx = x * inv;
  gy = y * inv;
}

// One channel's loads for a lane holding R vertically adjacent pixels:
// f0 column rows y0-1 .. y0+R (f[j] = row y0-1+j) and the f1 taps of each pixel.
template <int R>
struct ChanLoadsR {
  float f[R + 2];
  Gather4 g[R];
};
// Channel-quad layout (DPFT_FEATURES_C4): one 16-byte load per row / tap carries
// 4 channels.  t[r][0..3] = taps (x0, y0), (x0 + 1, y0), (x0, y1), (x0 + 1, y1)
// of the pair bases (see gather4).
template <int R>
struct QuadLoadsR {
  f32x4 f[R + 2];
  f32x4 t[R][4];
};

// ============================================================ ICP term (combine_ICP)
// Point-to-plane residual and inverse Jacobian of one pixel, ScaleNet('None')
// weight applied (algorithms.py:916-997, 668-689; geometry.py:1129-1136).
// Frame 1's normal map is pose-independent and comes from icp_normals_kernel, interleaved
// with frame 1's depth: one 16-byte [nx, ny, nz, depth1] element per pixel, so a tap is
// one load instead of four scalar gathers (same values, same arithmetic: same bits).
struct IcpTerm {
  float J[6];  // w * J (already the reference's negated, sigma-normalised J)
  float r;     // w * r (1e-6 * w where occluded)
  bool occ;
};

// The term in three parts, so that the marching kernel can issue the normal-map taps before
// the pixel's IC normal-equation update and consume them after it (that arithmetic then
// covers part of the loads' latency): icp_geo (projection, in-view test, taps: pose and
// depth0 only), icp_load (the four tap loads), icp_term (the rest).
struct IcpGeo {
  float V0x, V0y, V0z, Px, Py, Pz;
  bool inview;
  Taps tp;
  int x0, x1, y0, y1;
};
struct IcpTaps {
  f32x4 q00, q01, q10, q11;
};

__device__ __forceinline__ IcpGeo icp_geo(float xr, float yr, float d0, const float* __restrict__ Rm,
                                          const float* __restrict__ tv, float fx, float fy, float cx, float cy, int H,
                                          int W, const float* rs = nullptr) {
#pragma clang fp contract(off)
  IcpGeo g;
  // vertex0 = [px, py, 1] * depth0; P = R V0 + t (CPU bmm order, then + t)
  g.V0x = xr * d0;
  g.V0y = yr * d0;
  g.V0z = d0;
  g.Px = __builtin_fmaf(Rm[2], g.V0z, __builtin_fmaf(Rm[1], g.V0y, Rm[0] * g.V0x)) + tv[0];
  g.Py = __builtin_fmaf(Rm[5], g.V0z, __builtin_fmaf(Rm[4], g.V0y, Rm[3] * g.V0x)) + tv[1];
  g.Pz = __builtin_fmaf(Rm[8], g.V0z, __builtin_fmaf(Rm[7], g.V0y, Rm[6] * g.V0x)) + tv[2];
  const float u = (g.Px / g.Pz) * fx + cx;
  const float v = (g.Py / g.Pz) * fy + cy;
  g.inview = (u > 0.0f) && (u < (float)(W - 1)) && (v > 0.0f) && (v < (float)(H - 1));
  // (the taps are clamped into the image whatever u, v are -- NaN included -- so the loads
  // below stay in bounds on every lane)
  g.tp = rs ? make_taps_xy<true>(u, v, H, W, g.x0, g.x1, g.y0, g.y1, rs)
            : make_taps_xy<false>(u, v, H, W, g.x0, g.x1, g.y0, g.y1);
  return g;
}

__device__ __forceinline__ IcpTaps icp_load(const IcpGeo& g, const f32x4* __restrict__ nd1) {
  return IcpTaps{nd1[g.tp.o00], nd1[g.tp.o01], nd1[g.tp.o10], nd1[g.tp.o11]};
}

// The tap vertices' normalised coordinates (x - cx) / fx of the tap columns x0, x1 and
// (y - cy) / fy of the rows y0, y1 (geometry.py:1129-1136 on the tap pixels).
struct IcpTapXY {
  float px0, px1, py0, py1;
};
__device__ __forceinline__ IcpTapXY icp_tap_xy(const IcpGeo& g, float fx, float fy, float cx, float cy) {
#pragma clang fp contract(off)
  return IcpTapXY{((float)g.x0 - cx) / fx, ((float)g.x1 - cx) / fx, ((float)g.y0 - cy) / fy, ((float)g.y1 - cy) / fy};
}

__device__ __forceinline__ IcpTerm icp_term(const IcpGeo& g, const IcpTaps& q, const IcpTapXY& n, float d0,
                                            const float* __restrict__ Rm, bool mask0_bg,
                                            const uint8_t* __restrict__ m1b, float wgt) {
#pragma clang fp contract(off)
  const Taps& tp = g.tp;
  // vertex1 sampled: the vertex map at the four taps, then the sampler's chain
  const float a = q.q00.w, b = q.q01.w, c = q.q10.w, d = q.q11.w;
  const float px0 = n.px0, px1 = n.px1, py0 = n.py0, py1 = n.py1;
  const float V1x = bil4(px0 * a, px1 * b, px0 * c, px1 * d, tp);
  const float V1y = bil4(py0 * a, py0 * b, py1 * c, py1 * d, tp);
  const float V1z = bil4(a, b, c, d, tp);
  const float Nx = bil4(q.q00.x, q.q01.x, q.q10.x, q.q11.x, tp), Ny = bil4(q.q00.y, q.q01.y, q.q10.y, q.q11.y, tp);
  const float Nz = bil4(q.q00.z, q.q01.z, q.q10.z, q.q11.z, tp);
  const float Dx = g.Px - V1x, Dy = g.Py - V1y, Dz = g.Pz - V1z;
  // ||diff|| > 0.1 (936-940) as a test of the squared norm against the largest float whose
  // correctly rounded square root is <= 0.1f (0x3c23d70b): sqrt is monotonic, so the two tests
  // agree on every input (checked exhaustively around the threshold), without the IEEE
  // square-root sequence
  bool occ = !g.inview || ((Dx * Dx + Dy * Dy) + Dz * Dz > __uint_as_float(0x3c23d70bu)) || mask0_bg;
  if (m1b) occ = occ || !(bil_u8(m1b, tp) > 0.0f);
  float r = (Nx * Dx + Ny * Dy) + Nz * Dz;
  // n = N1w^T R ; J = [n x V0, -n]
  const float n0 = __builtin_fmaf(Nz, Rm[6], __builtin_fmaf(Ny, Rm[3], Nx * Rm[0]));
  const float n1 = __builtin_fmaf(Nz, Rm[7], __builtin_fmaf(Ny, Rm[4], Nx * Rm[1]));
  const float n2 = __builtin_fmaf(Nz, Rm[8], __builtin_fmaf(Ny, Rm[5], Nx * Rm[2]));
  // stereo-model sigma with the reference's hard-coded TUM constants (975-997).  Only the
  // divisions above feed discrete tests (the in-view test and the taps: X / Z, Y / Z; the
  // ||diff|| > 0.1 occlusion: the tap vertices) and stay op for op.  These only scale
  // continuous values: the constants are folded (depth / 525 * 5.5 -> depth * (5.5 / 525),
  // depth^2 * 0.4 / (525 * 1.2) -> depth^2 * (0.4 / 630)) and the seven divisions by
  // sigma_icp + 1e-8 (965-966) are one reciprocal and seven products (within a few ulp of
  // the quotients; the JtJ / JtR bounds are 1e-5 / 1e-4 relative)
  constexpr float kSxy = 5.5f / 525.0f, kSz = 0.4f / (525.0f * 1.2f);
  const float sxy = d0 * kSxy;
  const float sz = (d0 * d0) * kSz;
  const float cov = (((n0 * sxy) * sxy) * n0 + ((n1 * sxy) * sxy) * n1) + ((n2 * sz) * sz) * n2;
  // w / sigma (the ScaleNet weight folded in) by the hardware square root and reciprocal
  // (1 ulp each, no IEEE division / sqrt sequences): continuous weights only
  const float rsig = wgt * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(cov + 1e-8f) + 1e-8f);
  IcpTerm o;
  o.J[0] = (n2 * g.V0y - n1 * g.V0z) * rsig;
  o.J[1] = (n0 * g.V0z - n2 * g.V0x) * rsig;
  o.J[2] = (n1 * g.V0x - n0 * g.V0y) * rsig;
  o.J[3] = n0 * rsig;
  o.J[4] = n1 * rsig;
  o.J[5] = n2 * rsig;
  o.r = occ ? 1e-6f * wgt : r * rsig;
  o.occ = occ;
  return o;
}

__device__ __forceinline__ IcpTerm icp_pixel(float xr, float yr, float d0, const float* __restrict__ Rm,
                                             const float* __restrict__ tv, float fx, float fy, float cx, float cy,
                                             int H, int W, const f32x4* __restrict__ nd1, bool mask0_bg,
                                             const uint8_t* __restrict__ m1b, float wgt) {
  const IcpGeo g = icp_geo(xr, yr, d0, Rm, tv, fx, fy, cx, cy, H, W);
  return icp_term(g, icp_load(g, nd1), icp_tap_xy(g, fx, fy, cx, cy), d0, Rm, mask0_bg, m1b, wgt);
}

// Frame-1 normal map of one level (algorithms.py:2148-2172): vertex map
// (geometry.py:1129-1136), unnormalised replicate-padded Sobel, cross product,
// / (|n| + 1e-8), zero where depth equals the batch-global min or max; stored as
// [B][H][W] x [nx, ny, nz, depth1] (the depth beside its normal for icp_pixel's taps).
// `dext`: order-encoded (min, max) word pairs, one per independent batch of `group` pairs
// (DPFT_GROUP; group = B: the call is one batch, the reference's batch-global extrema).
// One wave per (pair, 62-column strip, run of `rpr` rows), marching down its run: lane l
// holds column 62 s - 1 + l (clamped: replicate padding) and keeps the vertices of rows
// y - 1, y, y + 1 in registers, so each depth row is loaded and turned into vertices once
// per run (one column division per lane, one row division per row) instead of nine
// vertices -- eighteen divisions, nine loads -- per pixel; the neighbour columns' vertices
// come from DPP lane shifts (as the marching kernel's Sobel).  The same IEEE operations on
// the same operands as per-pixel vertices, bit for bit.  Lanes 1 .. 62 store.  (One
// short-lived wave per pixel row was launch-bound: 375 -> 201 us at level 0 of 128 pairs.)
// Runs of up to 16 rows, shorter where that leaves fewer than 16 k waves (coarse levels).
// Every product and sum is rounded as written (no contraction), so the map does not depend
// on how the compiler schedules this code.
__host__ __device__ inline int nrm_rows(int B, int H, int W) {
  const long cols = (long)B * H * ((W + kTileOut - 1) / kTileOut);
  return (int)(cols >= 16L * 16384 ? 16 : cols >= 2L * 16384 ? cols / 16384 : 2);
}
__global__ __launch_bounds__(kThreads) void icp_normals_kernel(const float* __restrict__ depth, const float* __restrict__ K,
                                                               int B, int H, int W, const uint32_t* __restrict__ dext,
                                                               int group, f32x4* __restrict__ nrm) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int rpr = nrm_rows(B, H, W);
  const int strips = (W + kTileOut - 1) / kTileOut, runs = (H + rpr - 1) / rpr;
  const long unit = (long)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);  // (b, run, strip), strip fastest
  if (unit >= (long)B * runs * strips) return;  // wave-uniform
  const int s = (int)(unit % strips);
  const long br = unit / strips;
  const int b = (int)(br / runs), y0 = (int)(br - (long)b * runs) * rpr, y1 = min(y0 + rpr, H);
  const int HW = H * W;
  dext += 2 * (b / group);
  const float dmin = dec_ord(dext[0]), dmax = dec_ord(dext[1]);
  const float fx = K[4 * b + 0], fy = K[4 * b + 1], cx = K[4 * b + 2], cy = K[4 * b + 3];
  const float* db = depth + (size_t)b * HW;
  const int x = s * kTileOut - 1 + lane, xx = min(max(x, 0), W - 1);
  const bool out = lane >= 1 && lane <= kTileOut && x < W;
  const float xr = ((float)xx - cx) / fx;
  // vertices of one row at this lane's column and its two neighbours: [dx][xyz]
  auto row = [&](int y, float (&V)[3][3]) {
    const int yy = min(max(y, 0), H - 1);
    const float dd = db[yy * W + xx];
    V[1][0] = xr * dd;
    V[1][1] = (((float)yy - cy) / fy) * dd;
    V[1][2] = dd;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      V[0][c] = lane_from_left(V[1][c]);
      V[2][c] = lane_from_right(V[1][c]);
    }
  };
  float Vt[3][3], Vm[3][3], Vb[3][3];  // rows y - 1, y, y + 1
  row(y0 - 1, Vt);
  row(y0, Vm);
  for (int y = y0; y < y1; ++y) {
    row(y + 1, Vb);
    float gx[3], gy[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      gx[c] = ((Vt[2][c] - Vt[0][c]) + 2.0f * (Vm[2][c] - Vm[0][c])) + (Vb[2][c] - Vb[0][c]);
      gy[c] = ((Vb[0][c] - Vt[0][c]) + 2.0f * (Vb[1][c] - Vt[1][c])) + (Vb[2][c] - Vt[2][c]);
    }
    if (out) {
      const float n[3] = {gx[1] * gy[2] - gx[2] * gy[1], gx[2] * gy[0] - gx[0] * gy[2], gx[0] * gy[1] - gx[1] * gy[0]};
      const float mag = sqrtf((n[0] * n[0] + n[1] * n[1]) + n[2] * n[2]) + 1e-8f;
      const float d = Vm[1][2];
      nrm[(size_t)b * HW + (size_t)y * W + x] = (d == dmin || d == dmax) ? f32x4{0.0f, 0.0f, 0.0f, d}
                                                                          : f32x4{n[0] / mag, n[1] / mag, n[2] / mag, d};
    }
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        Vt[k][c] = Vm[k][c];
        Vm[k][c] = Vb[k][c];
      }
  }
}

// combine_ICP on the channel-quad path: the point-to-plane term's normal equations in a pass
// of their own (algorithms.py:916-997, 668-689), kIcpSub records per reduce workgroup slot
// (the reduce launch's B x nbpp), which pair_reduce2 adds to that slot's reduce record:
// workgroup (jb, u) of pair b takes pixels [HW s / (nbpp S), HW (s + 1) / (nbpp S)),
// s = jb S + u.  S workgroups per slot (p.fin.icp_sub, up to kIcpSub where a level has the
// pixels for it): at level 0 one workgroup per slot leaves two waves per SIMD, latency-bound
// (252 us per 64-pair launch; four: ...).  The term needs no feature
// bytes (depth0, the normal map's taps, the masks: 8 B per pixel of HBM plus cached taps), so
// the reduce launch keeps the U_IC kernel's registers -- the cross-row prefetch and the ring
// depth of the fused ICP kernel did not fit two waves per SIMD.  The
// pixel's normalised coordinates are the marching kernel's (norm_coord: the same IEEE
// operations), its contribution the fused kernel's (same icp_pixel, same weight); only the
// fp32 summation grouping differs.
__global__ __launch_bounds__(kThreads) void icp_records_kernel(IterParams p, float* __restrict__ out) {
  __shared__ float red[4][28];
  __shared__ float nxy[kIcpTab];  // (x - cx) / fx of the W columns, then (y - cy) / fy of the H rows
  const int kb = blockIdx.x, nsub = p.nbpp * p.fin.icp_sub, b = kb / nsub, sb = kb - b * nsub;
  const int W = p.W, H = p.H, HW = H * W;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float fx = p.K[4 * b + 0], fy = p.K[4 * b + 1], cx = p.K[4 * b + 2], cy = p.K[4 * b + 3];
  float Rm[9], tv[3];
#pragma unroll
  for (int k = 0; k < 9; ++k) Rm[k] = p.R[9 * b + k];
#pragma unroll
  for (int k = 0; k < 3; ++k) tv[k] = p.t[3 * b + k];
  // the pair's normalised coordinates once per workgroup (the same IEEE operations as
  // norm_coord: the same bits), read for the pixel and for its four tap vertices
  const bool tab = W + H <= kIcpTab;
  if (tab) {
    for (int j = tid; j < W + H; j += kThreads) nxy[j] = j < W ? norm_coord(j, cx, fx) : norm_coord(j - W, cy, fy);
    __syncthreads();
  }
  // the tap computation's divisors' reciprocals (make_taps_xy: exact division by a constant,
  // only for the image sizes it is verified for, p.rc_taps; else the IEEE division)
  const float rsxy[2] = {1.0f / ((float)(W - 1) * 0.5f), 1.0f / ((float)(H - 1) * 0.5f)};
  const float* d0b = p.depth0 + (size_t)b * HW;
  const uint8_t* m0b = p.mask0 ? p.mask0 + (size_t)b * HW : nullptr;
  const uint8_t* m1b = p.mask1 ? p.mask1 + (size_t)b * HW : nullptr;
  const f32x4* nd1 = p.nrm1 + (size_t)b * HW;
  const int beg = (int)(((long)HW * sb) / nsub), end = (int)(((long)HW * (sb + 1)) / nsub);
  float acc[27];
#pragma unroll
  for (int i = 0; i < 27; ++i) acc[i] = 0.f;
  // the pixel loop, instantiated with and without the table and div_const (no per-use branches)
  auto pixels = [&](auto table, auto rc) {
    constexpr bool TAB = decltype(table)::value, RC = decltype(rc)::value;
    auto ncx = [&](int x) { return TAB ? nxy[x] : norm_coord(x, cx, fx); };
    auto ncy = [&](int y) { return TAB ? nxy[W + y] : norm_coord(y, cy, fy); };
    // software-pipelined: pixel k + 1's depth0, geometry and normal-map taps are issued
    // before pixel k's term (two stages, A / B registers alternating: no loop-carried
    // copies); past the range the loads are clamped to its last pixel and not accumulated
    if (end <= beg) return;
    struct Stage {
      IcpGeo g;
      IcpTaps q;
      float d0;
      bool m0;
    };
    // depth0 one pixel further ahead (`dq`): loaded when the pixel before it is issued, so
    // the geometry and the tap loads of an issue wait on no load (the pass is bound by this
    // dependent chain, not by its VALU: level-0 iteration 2285 -> 2255 us, +0.9 % for cfg5)
    auto ld0 = [&](int pix) { return d0b[min(pix, end - 1)]; };
    auto issue = [&](Stage& S, int pix, int x, int y, float d0) {
      const int pc = min(pix, end - 1);
      S.m0 = m0b ? (m0b[pc] != 0) : true;
      S.d0 = d0;
      S.g = icp_geo(ncx(x), ncy(min(y, H - 1)), S.d0, Rm, tv, fx, fy, cx, cy, H, W, RC ? rsxy : nullptr);
      S.q = icp_load(S.g, nd1);
    };
    auto term = [&](const Stage& S) {
      const IcpTapXY n{ncx(S.g.x0), ncx(S.g.x1), ncy(S.g.y0), ncy(S.g.y1)};
      const IcpTerm ic = icp_term(S.g, S.q, n, S.d0, Rm, !S.m0, m1b, p.icp_w);
      int kq = 0;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
#pragma unroll
        for (int j = i; j < 6; ++j) acc[kq++] += ic.J[i] * ic.J[j];
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) acc[21 + i] += ic.J[i] * ic.r;
    };
    auto advance = [&](int& pix, int& x, int& y) {
      pix += kThreads;
      x += kThreads;
      while (x >= W) {
        x -= W;
        ++y;
      }
    };
    int pix = beg + tid, y = pix / W, x = pix - y * W;  // then advanced by kThreads without a division
    Stage A, Bs;
    float dq = ld0(pix);
    issue(A, pix, x, y, dq);
    dq = ld0(pix + kThreads);
    for (;;) {
      const int pa = pix;
      advance(pix, x, y);
      issue(Bs, pix, x, y, dq);
      dq = ld0(pix + kThreads);
      if (pa < end) term(A);
      if (pix >= end) break;
      const int pb = pix;
      advance(pix, x, y);
      issue(A, pix, x, y, dq);
      dq = ld0(pix + kThreads);
      if (pb < end) term(Bs);
      if (pix >= end) break;
    }
  };
  if (tab && p.rc_taps)
    pixels(std::true_type{}, std::true_type{});
  else if (tab)
    pixels(std::true_type{}, std::false_type{});
  else
    pixels(std::false_type{}, std::false_type{});
  // fixed-order reduction: wave butterflies, then the four waves in order
#pragma unroll
  for (int i = 0; i < 27; ++i) {
    float v = acc[i];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) red[wave][i] = v;
  }
  __syncthreads();
  if (tid < kIcpRec)
    out[(size_t)kb * kIcpRec + tid] = tid < 27 ? ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid] : 0.f;
}

// ============================================================ last-block finalize
__device__ __forceinline__ double wave_sum_d(double v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// Global (whole-batch) extrema of sigma_r over every record (all threads call).
__device__ void global_extrema(const float* rec, int nblocks, int imn, int imx, float& gmin, float& gmax) {
  __shared__ float sm[2][4];
  float mn = INFINITY, mx = -INFINITY;
  for (int k = threadIdx.x; k < nblocks; k += kThreads) {
    mn = fminf(mn, ld_ag(rec + (size_t)k * kRec + imn));
    mx = fmaxf(mx, ld_ag(rec + (size_t)k * kRec + imx));
  }
  for (int off = 32; off > 0; off >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, off));
    mx = fmaxf(mx, __shfl_xor(mx, off));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    sm[0][wave] = mn;
    sm[1][wave] = mx;
  }
  __syncthreads();
  gmin = fminf(fminf(sm[0][0], sm[0][1]), fminf(sm[0][2], sm[0][3]));
  gmax = fmaxf(fmaxf(sm[1][0], sm[1][1]), fmaxf(sm[1][2], sm[1][3]));
}

// 1 / sqrt(x) in fp64: the hardware estimate plus two Newton steps (the estimate is good
// to ~2^-22, each step doubles the bits) -- a few dependent FMAs instead of the
// correctly rounded sqrt and divide sequences on the finalize's serial path.  x = 0 and
// x < 0 (a non-SPD pivot) give inf / NaN like 1 / sqrt(x).
__device__ __forceinline__ double rsqrt_d(double x) {
  double r = __builtin_amdgcn_rsq(x);
  if (!(x > 0.0) || isinf(x)) return r;
#pragma unroll
  for (int i = 0; i < 2; ++i) r = r * __builtin_fma(-0.5 * x * r, r, 1.5);
  return r;
}

// Solve (JtJ + 1e-6 tr(JtJ) I) xi = JtR in fp64 (algorithms.py:2094-2103: the
// damped matrix is SPD, so a fully unrolled register Cholesky replaces the
// reference's batched inverse) and apply the inverse-compositional update
// (algorithms.py:2035-2054, geometry.py:105-123, 163-185):
// R <- R Exp(-w), t <- R (-Exp(-w) v) + t.
// `diag_add` (optional): extra damping on the diagonal, H = JtJ + diag(diag_add) +
// 1e-6 tr(JtJ) I -- the residual-volume trial and learned-damping matrices of
// 'Direct-ResVol' (algorithms.py:1664-1691); the 1e-6 tr term is the reference's
// epsilon there and lev_mar_H's damping here.
__device__ void solve_and_update(const double* jtj_u, const double* jtr, float* Rp, float* tp,
                                 const double* diag_add = nullptr) {
  double A[6][6];
  int k = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = i; j < 6; ++j) {
      A[i][j] = jtj_u[k];
      A[j][i] = jtj_u[k];
      ++k;
    }
  const double tr = ((((A[0][0] + A[1][1]) + A[2][2]) + A[3][3]) + A[4][4]) + A[5][5];
#pragma unroll
  for (int i = 0; i < 6; ++i) A[i][i] = (diag_add ? A[i][i] + diag_add[i] : A[i][i]) + 1e-6 * tr;
  double L[6][6], invd[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double dj = A[j][j];
#pragma unroll
    for (int m = 0; m < j; ++m) dj -= L[j][m] * L[j][m];
    invd[j] = rsqrt_d(dj);  // 1 / L[j][j]
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double v = A[i][j];
#pragma unroll
      for (int m = 0; m < j; ++m) v -= L[i][m] * L[j][m];
      L[i][j] = v * invd[j];
    }
  }
  double z[6], xi[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double v = jtr[i];
#pragma unroll
    for (int m = 0; m < i; ++m) v -= L[i][m] * z[m];
    z[i] = v * invd[i];
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    double v = z[i];
#pragma unroll
    for (int m = i + 1; m < 6; ++m) v -= L[m][i] * xi[m];
    xi[i] = v * invd[i];
  }
  // dR = Exp(-w): Rodrigues, NaN at |w| = 0 exactly as the reference.
  const double w0 = -xi[0], w1 = -xi[1], w2 = -xi[2];
  const double th2 = w0 * w0 + w1 * w1 + w2 * w2;
  const double ith = rsqrt_d(th2);  // inf at |w| = 0: k = NaN, as the reference's w / |w|
  const double th = th2 * ith;
  const double k0 = w0 * ith, k1 = w1 * ith, k2 = w2 * ith;
  const double Kx[9] = {0.0, -k2, k1, k2, 0.0, -k0, -k1, k0, 0.0};
  double sn, cs;
  sincos(th, &sn, &cs);
  const double cs1 = 1.0 - cs;
  double dR[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const double kk = Kx[3 * i] * Kx[j] + Kx[3 * i + 1] * Kx[3 + j] + Kx[3 * i + 2] * Kx[6 + j];
      dR[3 * i + j] = ((i == j) ? 1.0 : 0.0) + Kx[3 * i + j] * sn + kk * cs1;
    }
  double dt[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) dt[i] = -(dR[3 * i] * xi[3] + dR[3 * i + 1] * xi[4] + dR[3 * i + 2] * xi[5]);
  double R0[9], t0[3];
#pragma unroll
  for (int i = 0; i < 9; ++i) R0[i] = Rp[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) t0[i] = tp[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      Rp[3 * i + j] = (float)(R0[3 * i] * dR[j] + R0[3 * i + 1] * dR[3 + j] + R0[3 * i + 2] * dR[6 + j]);
    tp[i] = (float)(R0[3 * i] * dt[0] + R0[3 * i + 1] * dt[1] + R0[3 * i + 2] * dt[2] + t0[i]);
  }
}

// Workgroup-wide min / max of two floats (all threads call; result in all threads).
__device__ void block_minmax2(float& mn_a, float& mx_a, float& mn_b, float& mx_b) {
  __shared__ float sm[4][4];
  for (int off = 32; off > 0; off >>= 1) {
    mn_a = fminf(mn_a, __shfl_xor(mn_a, off));
    mx_a = fmaxf(mx_a, __shfl_xor(mx_a, off));
    mn_b = fminf(mn_b, __shfl_xor(mn_b, off));
    mx_b = fmaxf(mx_b, __shfl_xor(mx_b, off));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();  // sm may still be read by a previous call
  if (lane == 0 && wave < 4) {  // workgroups wider than kThreads: the extra waves carry no data
    sm[0][wave] = mn_a;
    sm[1][wave] = mx_a;
    sm[2][wave] = mn_b;
    sm[3][wave] = mx_b;
  }
  __syncthreads();
  mn_a = fminf(fminf(sm[0][0], sm[0][1]), fminf(sm[0][2], sm[0][3]));
  mx_a = fmaxf(fmaxf(sm[1][0], sm[1][1]), fmaxf(sm[1][2], sm[1][3]));
  mn_b = fminf(fminf(sm[2][0], sm[2][1]), fminf(sm[2][2], sm[2][3]));
  mx_b = fmaxf(fmaxf(sm[3][0], sm[3][1]), fmaxf(sm[3][2], sm[3][3]));
}

// The pair record as pair_reduce2 stores it, kept in LDS too: a batch of one pair (q.group == 1)
// is solved from it by the same workgroup, without the record's round trip through L2.
__device__ __forceinline__ double* pair_rec_lds() {
  __shared__ double rec[kPRec];
  return rec;
}

// Run by the workgroup that completes the last pair: batch-global truncated-sigma
// extrema over the pair records, corrections, then one thread per pair solves and
// updates its pose (algorithms.py:2017-2103).
// `get(b, i)` reads field i of pair b's fp64 record (kPRec layout).
template <class Get>
__device__ void finalize_batch_from(const FinParams& q, Get get) {
  const bool tru = (q.flags & DPFT_REMOVE_TRU_SIGMA) != 0;
  const int B = q.B;
  float gmin = INFINITY, gmax = -INFINITY, u0 = INFINITY, u1 = -INFINITY;
  if (tru) {
    for (int b = threadIdx.x; threadIdx.x < kThreads && b < B; b += kThreads) {
      gmin = fminf(gmin, (float)get(b, P_MN_ALL));
      gmax = fmaxf(gmax, (float)get(b, P_MX_ALL));
    }
    block_minmax2(gmin, gmax, u0, u1);
  }
  for (int b = threadIdx.x; threadIdx.x < kThreads && b < B; b += kThreads) {
    double sv[28];
#pragma unroll
    for (int k = 0; k < 28; ++k) sv[k] = get(b, P_S + k);
    if (tru) {
      if ((float)get(b, P_MN0) == gmin)
#pragma unroll
        for (int k = 0; k < 7; ++k) sv[21 + k] += get(b, P_CMN + k);
      if (gmax != gmin && (float)get(b, P_MX0) == gmax)
#pragma unroll
        for (int k = 0; k < 7; ++k) sv[21 + k] += get(b, P_CMX + k);
    }
    bool finite = true;
#pragma unroll
    for (int k = 0; k < 27; ++k) finite = finite && isfinite(sv[k]);
    if (!finite && q.status) atomicOr(q.status, DPFT_STATUS_NONFINITE);
    if (q.jtj_out) {
      int k = 0;
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = r; c < 6; ++c) {
          q.jtj_out[36 * b + 6 * r + c] = (float)sv[k];
          q.jtj_out[36 * b + 6 * c + r] = (float)sv[k];
          ++k;
        }
    }
    if (q.jtr_out)
#pragma unroll
      for (int k = 0; k < 6; ++k) q.jtr_out[6 * b + k] = (float)sv[21 + k];
    if (q.invalid_out) q.invalid_out[b] = (int32_t)sv[27];
    if (!q.no_update) solve_and_update(sv, sv + 21, q.R + 9 * b, q.t + 3 * b);
  }
}
// (Loading each pair record in one burst of 16-byte sc1 loads before the extrema are
// known measured 6 us SLOWER per finalize than these field loads: not adopted.)
__device__ void finalize_batch(const FinParams& q) {
  if (q.B > kThreads) {
    finalize_batch_from(q, [&](int b, int i) { return ld_ag(q.prec + (size_t)b * kPRec + i); });
    return;
  }
  // thread b: every field of pair b's record up front (independent 8-byte sc1 loads, one
  // round trip), then the same computation from registers
  double r[46];
  if ((int)threadIdx.x < q.B) {
    const double* pr = q.prec + (size_t)threadIdx.x * kPRec;
#pragma unroll
    for (int i = 0; i < 46; ++i) r[i] = ld_ag(pr + i);
  }
  finalize_batch_from(q, [&](int, int i) { return r[i]; });
}

// Called by the workgroup that reduced pair b: the last of pair b's batch to finish
// (DPFT_GROUP: q.group pairs per independent batch, else the whole call) solves that
// batch -- its own truncated-sigma extrema, as if it had been a call of its own.
__device__ bool finalize_group(const FinParams& q, int b) {
  const int g = b / q.group, b0 = g * q.group;
  if (q.group == 1) {  // a batch of one pair (B = 1): this workgroup, which reduced the pair, solves it
    __syncthreads();     // from the pair record's LDS copy (pair_reduce2; the same values as stored)
    FinParams qg = q;
    qg.B = 1;
    qg.R = q.R ? q.R + 9 * b : nullptr;
    qg.t = q.t ? q.t + 3 * b : nullptr;
    qg.jtj_out = q.jtj_out ? q.jtj_out + 36 * b : nullptr;
    qg.jtr_out = q.jtr_out ? q.jtr_out + 6 * b : nullptr;
    qg.invalid_out = q.invalid_out ? q.invalid_out + b : nullptr;
    const double* lr = pair_rec_lds();
    double r[46];
    if (threadIdx.x == 0)
#pragma unroll
      for (int i = 0; i < 46; ++i) r[i] = lr[i];
    finalize_batch_from(qg, [&](int, int i) { return r[i]; });
    return true;
  }
  if (!block_is_last(q.done_cnt + g, 1u, (uint32_t)q.group)) return false;
  FinParams qg = q;
  qg.B = q.group;
  qg.prec = q.prec + (size_t)b0 * kPRec;
  qg.R = q.R ? q.R + 9 * b0 : nullptr;
  qg.t = q.t ? q.t + 3 * b0 : nullptr;
  qg.jtj_out = q.jtj_out ? q.jtj_out + 36 * b0 : nullptr;
  qg.jtr_out = q.jtr_out ? q.jtr_out + 6 * b0 : nullptr;
  qg.invalid_out = q.invalid_out ? q.invalid_out + b0 : nullptr;
  finalize_batch(qg);
  return true;
}

// Wave min / max trees (fixed order), every value moved before each step's wait.
// v[0], v[1]: min; v[2], v[3]: max
__device__ __forceinline__ void wave_minmax4(float (&v)[4]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int addr = (lane ^ off) << 2;
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v[i])));
    v[0] = fminf(v[0], o[0]);
    v[1] = fminf(v[1], o[1]);
    v[2] = fmaxf(v[2], o[2]);
    v[3] = fmaxf(v[3], o[3]);
  }
}

// Run by the last workgroup of pair b: its nbpp workgroup records -> one fp64 pair
// record (kPRec layout) in one load round trip.  Thread t holds record t (16-byte sc1
// loads: agent-coherent, as the records were stored); records t + 256, ... (pairs
// with more than 256 workgroups) are folded into it in record order (sums in fp32,
// extrema by ext_merge's ties-add rule).  The pair's sigma_r extrema decide which
// records' truncated-sigma corrections count; then quad sums by DPP and an LDS
// transpose reduce the 42 fields (28 without truncated sigma) column by column in
// fp64.  Fixed order throughout: deterministic for any finishing order.  `sc`: LDS the
// launch no longer needs, >= kFinScratch floats.
__device__ void pair_reduce2(const FinParams& q, int b, float* sc) {
  const bool tru = (q.flags & DPFT_REMOVE_TRU_SIGMA) != 0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = q.nbpp;
  const Rsrc rr = rsrc(q.rec + (size_t)b * n * kRec, (uint32_t)((size_t)n * kRec * sizeof(float)));
  float f[48];
#pragma unroll
  for (int i = 0; i < 48; ++i) f[i] = 0.f;
  f[R_MN_ALL] = f[R_MN0] = INFINITY;
  f[R_MX_ALL] = f[R_MX0] = -INFINITY;
  const int ns = q.icp_sub;
  const Rsrc ri = rsrc(q.icp_rec ? q.icp_rec + (size_t)b * n * ns * kIcpRec : q.rec,
                       q.icp_rec ? (uint32_t)((size_t)n * ns * kIcpRec * sizeof(float)) : 0u);
  for (int k = tid; k < n; k += kThreads) {
    f32x4 v[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) v[j] = llvm_buf_load_f32x4(rr, k * kRec * 4 + 16 * j, 0, kAuxSc1);
    if (q.icp_rec) {  // the point-to-plane term's normal equations of the same record slot
      for (int u = 0; u < ns; ++u)
#pragma unroll
        for (int j = 0; j < 7; ++j) v[j] += llvm_buf_load_f32x4(ri, (k * ns + u) * kIcpRec * 4 + 16 * j, 0, kAuxSc1);
    }
    const float* g = reinterpret_cast<const float*>(v);
    if (k == tid) {
#pragma unroll
      for (int i = 0; i < 48; ++i) f[i] = g[i];
      if (!tru) {
        f[R_MN_ALL] = f[R_MN0] = INFINITY;
        f[R_MX_ALL] = f[R_MX0] = -INFINITY;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 28; ++i) f[i] += g[i];
      if (tru) {
        Extremum e;
        e.all = f[R_MN_ALL];
        e.v0 = f[R_MN0];
        e.n = f[R_NMN];
#pragma unroll
        for (int i = 0; i < 6; ++i) e.c[i] = f[R_CMN + i];
        ext_merge<true>(e, g[R_MN_ALL], g[R_MN0], g + R_CMN, g[R_NMN]);
        f[R_MN_ALL] = e.all;
        f[R_MN0] = e.v0;
        f[R_NMN] = e.n;
#pragma unroll
        for (int i = 0; i < 6; ++i) f[R_CMN + i] = e.c[i];
        e.all = f[R_MX_ALL];
        e.v0 = f[R_MX0];
        e.n = f[R_NMX];
#pragma unroll
        for (int i = 0; i < 6; ++i) e.c[i] = f[R_CMX + i];
        ext_merge<false>(e, g[R_MX_ALL], g[R_MX0], g + R_CMX, g[R_NMX]);
        f[R_MX_ALL] = e.all;
        f[R_MX0] = e.v0;
        f[R_NMX] = e.n;
#pragma unroll
        for (int i = 0; i < 6; ++i) f[R_CMX + i] = e.c[i];
      }
    }
  }
  // pair extrema of sigma_r first (which records' corrections count)
  float ex[4] = {f[R_MN_ALL], f[R_MN0], f[R_MX_ALL], f[R_MX0]};
  if (tru) {
    wave_minmax4(ex);
    float* scf = sc;
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < 4; ++i) scf[4 * wave + i] = ex[i];
    __syncthreads();
    ex[0] = fminf(fminf(scf[0], scf[4]), fminf(scf[8], scf[12]));
    ex[1] = fminf(fminf(scf[1], scf[5]), fminf(scf[9], scf[13]));
    ex[2] = fmaxf(fmaxf(scf[2], scf[6]), fmaxf(scf[10], scf[14]));
    ex[3] = fmaxf(fmaxf(scf[3], scf[7]), fmaxf(scf[11], scf[15]));
    __syncthreads();  // scf is reused below
  }
  // fields in the pair-record order: 28 sums, then the 7 + 7 corrections (masked)
  const bool use_mn = f[R_MN0] == ex[1], use_mx = f[R_MX0] == ex[3];
  auto field = [&](int i) -> float {
    if (i < 28) return f[i];
    if (i < 35) return use_mn ? f[R_CMN + (i - 28)] : 0.f;  // R_CMN + 6 == R_NMN
    return use_mx ? f[R_CMX + (i - 35)] : 0.f;              // R_CMX + 6 == R_NMX
  };
  const int nf = tru ? 42 : 28;
  // quad sums by DPP (xor 1, then xor 2: ((r0 + r1) + (r2 + r3)) in every lane of the
  // quad), then the 64 quad rows transposed through LDS ([field][65]: conflict-free
  // columns) and summed per field in fp64, row order -- no cross-lane shuffle chains
  float* L = sc;
#pragma unroll
  for (int i = 0; i < 42; ++i) {
    float v = field(i);
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xf, 0xf, true));  // quad_perm 1,0,3,2
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xf, 0xf, true));  // quad_perm 2,3,0,1
    if (i < nf && (tid & 3) == 0) L[i * 65 + (tid >> 2)] = v;
  }
  __syncthreads();
  double* pr = q.prec + (size_t)b * kPRec;
  double* lr = pair_rec_lds();
  if (tid < nf) {
    double v = 0.0;
    const float* col = L + tid * 65;
#pragma unroll 16
    for (int r = 0; r < 64; ++r) v += (double)col[r];
    const int fld = tid < 28 ? P_S + tid : tid < 35 ? P_CMN + (tid - 28) : P_CMX + (tid - 35);
    st_ag(pr + fld, v);
    lr[fld] = v;
  } else if (tid >= 64 && tid < 64 + 2 * 7 && !tru) {
    st_ag(pr + P_CMN + (tid - 64), 0.0);  // (P_CMX follows P_CMN)
    lr[P_CMN + (tid - 64)] = 0.0;
  } else if (tid >= 128 && tid < 132) {
    const int i = tid - 128, fld = i == 0 ? P_MN_ALL : i == 1 ? P_MN0 : i == 2 ? P_MX_ALL : P_MX0;
    st_ag(pr + fld, (double)ex[i]);
    lr[fld] = (double)ex[i];
  }
}


// Last workgroup of a residual launch: loss[b] = sum / (HW - #invalid)
// (algorithms.py:2119-2137).
__device__ void finalize_loss(const FinParams& q) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool tru = (q.flags & DPFT_REMOVE_TRU_SIGMA) != 0;
  float gmin = 0.f, gmax = 0.f;
  if (tru) global_extrema(q.rec, q.nblocks, L_MN_ALL, L_MX_ALL, gmin, gmax);
  const int B = q.nblocks / q.per_pair;
  for (int b = wave; b < B; b += 4) {
    double sum = 0.0, ninv = 0.0;
    for (int k = lane; k < q.per_pair; k += 64) {
      const float* r = q.rec + (size_t)(b * q.per_pair + k) * kRec;
      sum += ld_ag(r + L_SUM);
      ninv += ld_ag(r + L_NINV);
      if (tru) {
        if (ld_ag(r + L_MN0) == gmin) { sum -= ld_ag(r + L_LMN); ninv += ld_ag(r + L_NMN); }
        if (gmax != gmin && ld_ag(r + L_MX0) == gmax) { sum -= ld_ag(r + L_LMX); ninv += ld_ag(r + L_NMX); }
      }
    }
    sum = wave_sum_d(sum);
    ninv = wave_sum_d(ninv);
    if (lane == 0) q.loss_out[b] = (float)(sum / ((double)q.HW - ninv));
  }
}

// ============================================================ fused reduce kernel
// Loads of channel chunk k+1 are issued before chunk k's math; chunks go in
// (even, odd) pairs so each load set lives in fixed registers and no in-flight
// load is ever copied (a copy would force the wait the prefetch exists to avoid).
// Work split: a pair's level is tiles_x * row_groups tiles of 4 rows x 62
// columns, ordered (column strip, row group).  Each pair gets nbpp workgroups
// (B * nbpp ~ the device's resident capacity: no tail round) and workgroup j of
// pair b takes the contiguous tile range [n j / nbpp, n (j+1) / nbpp): one
// prologue / epilogue per workgroup, and consecutive tiles are vertically
// adjacent, so the halo rows of f0 / sigma0 are re-read from L2 right after
// their first use.  Workgroup k writes record slot k.
// MODE: 0 = U_IC (TrustRegionInverseWUncertainty), 1 = U_IC + combine_ICP,
//       2 = IC without uncertainty (TrustRegionBase, algorithms.py:23-139: sigma = 1,
//           J = Jf_x Jx + Jf_y Jy (1867-1882), occluded residual 1e-3 (1955)).
template <int CT, bool CS1, bool TRU, int MODE, bool C4>
__global__ __launch_bounds__(kThreads, 1) void ic_reduce_kernel(IterParams p) {
  constexpr bool ICP = MODE == 1, NOSIG = MODE == 2;
  static_assert(!C4 || CS1, "the channel-quad layout needs one sigma plane");
  constexpr int R = C4 ? ((CT > 0) ? 1 : kRPL4) : (CS1 ? kRPL : 1);  // rows per lane
  constexpr float kFill = NOSIG ? 1e-3f : 1e-6f;  // weighted residual of invalid pixels
  const int C = CT > 0 ? CT : p.C;
  __shared__ float lds_ext[TRU ? 2 * 7 : 1][kThreads];  // extremum corrections (6 + count), min then max
  __shared__ float red[4][kRec];
  constexpr bool kWin = C4 && CT > 0;  // channel-quad marching window (C = 16, 32)
  __shared__ f32x4 lds_win[kWin ? 4 : 1][kWin ? 2 * (CT / 4) * 64 : 1];  // used: 2 x NQW quads per wave
  // pair_reduce2 scratch where neither the window nor the extremum buffer is there to reuse
  __shared__ float fin_sc[(kWin || TRU) ? 1 : 28 * 65];
  static_assert(!kWin || sizeof(lds_win) >= kFinScratch * sizeof(float), "finalize scratch (window)");
  static_assert(!TRU || sizeof(lds_ext) >= kFinScratch * sizeof(float), "finalize scratch (extremum buffer)");

  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int W = p.W, H = p.H, HW = H * W;
  const int kb = pair_slot_remap(blockIdx.x, gridDim.x, p.nbpp, p.round_wg);
  const int b = kb / p.nbpp, jb = kb - b * p.nbpp;
  const int seg_begin = b * p.per_pair + (int)(((long)p.per_pair * jb) / p.nbpp);
  const int seg_end = b * p.per_pair + (int)(((long)p.per_pair * (jb + 1)) / p.nbpp);
  const int grp2 = 2 * (b / p.fin.group);  // this pair's batch: its sigma0 extrema
  const float g0min = TRU ? dec_ord(p.ext[grp2]) : 0.f, g0max = TRU ? dec_ord(p.ext[grp2 + 1]) : 0.f;
  const uint32_t planeB = (uint32_t)HW * 4u;
  const int nch = C4 ? C / 4 : (C + kCK - 1) / kCK;    // one unit = one channel quad / kCK channels
  const int nunits = (nch + kRing - 1) / kRing * kRing;  // units per step, padded to the ring (empty tail units)

  const float fx = p.K[4 * b + 0], fy = p.K[4 * b + 1], cx = p.K[4 * b + 2], cy = p.K[4 * b + 3];
  float Rm[9], tv[3];
#pragma unroll
  for (int k = 0; k < 9; ++k) Rm[k] = p.R[9 * b + k];
#pragma unroll
  for (int k = 0; k < 3; ++k) tv[k] = p.t[3 * b + k];

  const auto rf0 = rsrc(p.f0 + (size_t)b * C * HW, planeB * C);
  const auto rf1 = rsrc(p.f1 + (size_t)b * C * HW, planeB * C);
  const auto rs0 = rsrc(p.s0 + (size_t)b * p.Cs * HW, planeB * p.Cs);
  const auto rs1 = rsrc(p.s1 + (size_t)b * p.Cs * HW, planeB * p.Cs);
  const auto rd0 = rsrc(p.invD0 + (size_t)b * HW, planeB);
  const auto rd1 = rsrc(p.invD1 + (size_t)b * HW, planeB);
  const uint8_t* m0b = p.mask0 ? p.mask0 + (size_t)b * HW : nullptr;
  const uint8_t* m1b = p.mask1 ? p.mask1 + (size_t)b * HW : nullptr;

  float acc[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) acc[k] = 0.0f;
  float ninv = 0.0f;
  float mn_all = INFINITY, mn0 = INFINITY, mx_all = -INFINITY, mx0 = -INFINITY;
  if (TRU) {
#pragma unroll
    for (int k = 0; k < 14; ++k) lds_ext[k][tid] = 0.0f;
  }

  // tile -> (column strip, first row of this wave); rows past H are clamped for
  // the loads and skipped by the accumulation
  // Tile order.  Channel-quad layout: column-major, a workgroup walks DOWN a
  // 62-column strip, so the stencil / tap rows shared with the tile above are more
  // often still in this XCD's L2 (measured L0 fetch 1.05 GB vs 1.13 GB row-major,
  // 212 vs 217 us).  NCHW: row-major (column-major measured 12 % slower there).
  constexpr bool kColMajor = C4;
  auto tile_pos = [&](int i, int& xs, int& y) {
    const int local = i - b * p.per_pair;
    int tx, ty;
    if (kColMajor) {
      tx = local / p.row_groups;
      ty = local - tx * p.row_groups;
    } else {
      ty = local / p.tiles_x;
      tx = local - ty * p.tiles_x;
    }
    y = ty * p.rps + wave * R;
    xs = tx * kTileOut - 1 + lane;                  // this lane's image column (may be -1 or >= W)
  };
  // ---- per-tile frame: warp, taps, occlusion inputs, masks (geometry.py:291-350, algorithms.py:1999-2008)
  struct Frame {
    int y0, xc, colv;
    bool out_lane, skip;  // skip: wave-uniform, every row of this wave is past the image
    int rows[R + 2];      // byte offsets of rows y0-1 .. y0+R, replicate-clamped
    float d[R];
    Warp wp[R];
    Taps tp[R];           // only ob0 / ob1 are read after make_frame
    PairWeights pw[R];
    Gather4 gd1[R], gs1[R];
    bool m0[R];
    float m1[R];
    float s0r[R + 2];
  };
  auto load_d = [&](int it, float (&dv)[R]) {
    int xs, y0;
    tile_pos(it, xs, y0);
#pragma unroll
    for (int r = 0; r < R; ++r) dv[r] = bld(rd0, min(y0 + r, H - 1) * W * 4 + min(max(xs, 0), W - 1) * 4, 0);
  };
  // frame of tile `it` from its inverse depths; issues the frame's gathers (consumed by pixel_terms)
  // xyr: the normalised coordinates of the pixel when the caller has them (R == 1), else null
  auto make_frame_xy = [&](int xs, int y0, const float (&dv)[R], Frame& F, bool s0_rows, const float* xyr = nullptr) {
    F.y0 = y0;
    F.xc = min(max(xs, 0), W - 1);  // clamped: replicate padding of the stencil
    F.out_lane = (lane >= 1) && (lane <= kTileOut) && (xs < W);
    F.colv = F.xc * 4;
    F.skip = __builtin_amdgcn_readfirstlane(F.y0) >= H;
    if (F.skip) return;
#pragma unroll
    for (int j = 0; j < R + 2; ++j) F.rows[j] = min(max(F.y0 - 1 + j, 0), H - 1) * W * 4;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int yr = min(F.y0 + r, H - 1);
      F.d[r] = dv[r];
      F.wp[r] = xyr ? warp_point_n(xyr[0], xyr[1], dv[r], Rm, tv, fx, fy, cx, cy)
                    : warp_point(F.xc, yr, dv[r], Rm, tv, fx, fy, cx, cy);
      F.tp[r] = make_taps(F.wp[r].u, F.wp[r].v, H, W);
      F.pw[r] = pair_weights(F.tp[r]);
      F.gd1[r] = gather4(rd1, F.tp[r], 0);
      F.m0[r] = m0b ? (m0b[yr * W + F.xc] != 0) : true;
      F.m1[r] = m1b ? bil_u8(m1b, F.tp[r]) : 1.0f;
      if (CS1 && !NOSIG) F.gs1[r] = gather4(rs1, F.tp[r], 0);
    }
    if (CS1 && !NOSIG && s0_rows) {
#pragma unroll
      for (int j = 0; j < R + 2; ++j) F.s0r[j] = bld(rs0, F.colv, F.rows[j]);
    }
  };
  auto make_frame = [&](int it, const float (&dv)[R], Frame& F) {
    int xs, y0;
    tile_pos(it, xs, y0);
    make_frame_xy(xs, y0, dv, F, true);
  };

  // per-pixel occlusion / uncertainty terms of a frame (one sigma plane: before or after the channels)
  struct PixelTerms {
    bool invalid[R];
    float sr0[R], srmin[R], srmax[R], inv_s[R], kk[R], hx[R], hy[R];
  };
  auto pixel_terms = [&](const Frame& F, PixelTerms& T) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float d1w = bilp(F.gd1[r], F.pw[r]);
      const bool ok = (F.wp[r].iz > d1w - 0.1f) && (F.wp[r].u > 0.0f) && (F.wp[r].u < (float)W) &&
                      (F.wp[r].v > 0.0f) && (F.wp[r].v < (float)H);
      T.invalid[r] = !ok || !F.out_lane || !F.m0[r] || !(F.m1[r] > 0.0f);
      T.sr0[r] = T.srmin[r] = T.srmax[r] = 0.f;
      T.inv_s[r] = NOSIG ? 1.0f : 0.f;
      T.kk[r] = T.hx[r] = T.hy[r] = 0.f;
      if (CS1 && !NOSIG) {
        sobel_cols(F.s0r[r], F.s0r[r + 1], F.s0r[r + 2], T.hx[r], T.hy[r]);
        T.sr0[r] = bilp(F.gs1[r], F.pw[r]);
        T.srmin[r] = T.srmax[r] = T.sr0[r];
        const float s0m = F.s0r[r + 1];
        // sigma and 1 / sigma by the hardware square root and reciprocal (1 ulp each; only
        // continuous weights depend on them, no test does)
        const float sg = __builtin_amdgcn_sqrtf(T.sr0[r] * T.sr0[r] + s0m * s0m);
        T.inv_s[r] = __builtin_amdgcn_rcpf(sg);
        T.kk[r] = s0m * (T.inv_s[r] * T.inv_s[r] * T.inv_s[r]);
        if (TRU) T.invalid[r] = T.invalid[r] || (s0m == g0min) || (s0m == g0max);
      }
    }
  };

  // the seven per-pixel channel sums -> JtJ / JtR / invalid count / extremum corrections
  struct Sums {
    float Saa[R], Sab[R], Sbb[R], Sa[R], Sb[R], Sar[R], Sbr[R];
  };
  // d0q (combine_ICP, R == 1): depth0 of the pixel, loaded by the caller before the
  // pixel's epilogue (the marching path); null: loaded here
  auto finish_pixels = [&](const Frame& F, const PixelTerms& T, Sums& S, const float* d0q = nullptr) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (!F.out_lane || F.y0 + r >= H) continue;
      // IC tracker with a learned M-estimator: the pixel's weight scales its J^T W J and
      // J^T W r terms (wJ = weights * J, algorithms.py:71-76; JtR = J^T (weights * r), 1631-1632)
      const float wp = (NOSIG && p.wgt) ? p.wgt[(size_t)b * HW + (size_t)(F.y0 + r) * W + F.xc] : 1.0f;
      const float Sa = -S.Sa[r] * wp, Sb = -S.Sb[r] * wp, Sar = -S.Sar[r] * wp, Sbr = -S.Sbr[r] * wp;
      const float Saa = S.Saa[r] * wp, Sab = S.Sab[r] * wp, Sbb = S.Sbb[r] * wp;
      const bool invalid = T.invalid[r];
      // combine_ICP: the point-to-plane term's geometry and its four normal-map taps first,
      // so that the IC update below runs while they load
      IcpGeo icg{};
      IcpTaps icq{};
      float d0v = 0.f;
      if constexpr (ICP) {
        d0v = (R == 1 && d0q) ? *d0q : p.depth0[(size_t)b * HW + (F.y0 + r) * W + F.xc];
        icg = icp_geo(F.wp[r].xr, F.wp[r].yr, d0v, Rm, tv, fx, fy, cx, cy, H, W);
        icq = icp_load(icg, p.nrm1 + (size_t)b * HW);
      }
      float Jx[6], Jy[6];
      warp_jac(F.wp[r].xr, F.wp[r].yr, F.d[r], fx, fy, Jx, Jy);
      // weighted residual of invalid pixels is 1e-6 on every channel (algorithms.py:1982-1983)
      const float cA = invalid ? kFill * Sa : Sar;
      const float cB = invalid ? kFill * Sb : Sbr;
      float P[6], Qv[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        P[i] = Saa * Jx[i] + Sab * Jy[i];
        Qv[i] = Sab * Jx[i] + Sbb * Jy[i];
      }
      int kq = 0;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
#pragma unroll
        for (int j = i; j < 6; ++j) {
          acc[kq] += P[i] * Jx[j] + Qv[i] * Jy[j];
          ++kq;
        }
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) acc[21 + i] -= cA * Jx[i] + cB * Jy[i];
      ninv += invalid ? 1.0f : 0.0f;
      if (ICP) {  // JtWJ += (wJ)^T (wJ), JtR += (wJ)^T (w r)  (algorithms.py:668-689)
        const IcpTerm ic = icp_term(icg, icq, icp_tap_xy(icg, fx, fy, cx, cy), d0v, Rm, !F.m0[r], m1b, p.icp_w);
        int kq2 = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
#pragma unroll
          for (int j = i; j < 6; ++j) acc[kq2++] += ic.J[i] * ic.J[j];
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) acc[21 + i] += ic.J[i] * ic.r;
      }

      if (TRU) {
        mn_all = fminf(mn_all, T.srmin[r]);
        mx_all = fmaxf(mx_all, T.srmax[r]);
        const float sr0 = T.sr0[r];
        const bool le = sr0 <= mn0, ge = sr0 >= mx0;
        if (le || ge) {
          float corr[7];
          const float dA = invalid ? 0.0f : (1e-6f * Sa - Sar);
          const float dB = invalid ? 0.0f : (1e-6f * Sb - Sbr);
#pragma unroll
          for (int i = 0; i < 6; ++i) corr[i] = -(dA * Jx[i] + dB * Jy[i]);
          corr[6] = invalid ? 0.0f : 1.0f;
          if (le) {
            const bool reset = sr0 < mn0;
            mn0 = sr0;
#pragma unroll
            for (int i = 0; i < 7; ++i) lds_ext[i][tid] = (reset ? 0.0f : lds_ext[i][tid]) + corr[i];
          }
          if (ge) {
            const bool reset = sr0 > mx0;
            mx0 = sr0;
#pragma unroll
            for (int i = 0; i < 7; ++i) lds_ext[7 + i][tid] = (reset ? 0.0f : lds_ext[7 + i][tid]) + corr[i];
          }
        }
      }
    }
  };

  if constexpr (kWin) {
    // ---- channel-quad layout, row-marching register window.  Each WAVE owns a
    // contiguous run of (column strip, row) units of its pair, strip-major, and walks
    // it row by row keeping the f0 rows y - dir and y of every quad (and of sigma0) in
    // registers: per row and quad it loads only row y + dir of f0 plus the f1 taps,
    // so every f0 / sigma0 row comes from HBM once per band instead of three times
    // (the tile path re-reads the halo rows after L2 has dropped them).  Odd waves
    // march upwards, so the two waves that share a band boundary reach it at the same
    // time (at the start, or at the end) and its halo rows / tap rows hit in L2.
    // The per-pixel weights factor out of the channel sums exactly as on the tile path.
    constexpr int NQ = CT / 4;
    static_assert(CT % 4 == 0, "channel quads");
    const int U = p.tiles_x * H;
    constexpr int NQW = NQ;                            // every quad of a pixel in one wave
    const int band = jb * 4 + wave, nw = p.nbpp * 4;  // this wave's band, the pair's waves
    // Band sizes: the first half of a pair's waves belongs to the workgroups dispatched
    // first, which the oldest-first issue arbitration favours over the second
    // workgroup on the same CU; equal bands leave the second half running alone
    // (at half occupancy) for ~20 % of the launch.  Weights 64 + skew / 64 - skew.
    // n bands of a total of `len` units, weights 64 + skew for the first half, 64 - skew
    auto split_start = [&](int bnd, int n, int len) {
      const int h = n >> 1, sk = n >= 2 ? p.skew : 0;
      const long wsum = (long)(64 + sk) * min(bnd, h) + (long)(64 - sk) * max(bnd - h, 0);
      const long wtot = (long)(64 + sk) * h + (long)(64 - sk) * (n - h);
      return (int)(((long)len * wsum) / wtot);
    };
    // Grid split (kMarchGrid): K row bands x S strips, band = k * S + s, every strip cut
    // at the same rows.  A strip's 64 lanes read columns 62 s - 1 .. 62 s + 62, so the
    // 128-byte lines at a strip boundary belong to both strips (1.15x f0 lines per row);
    // with a common row cut the two waves read them within a row-step of each other (an
    // L2 hit for the second) instead of tens of microseconds apart.  Up to nw / 16 waves
    // may be left without a band (nw - K S); otherwise the strip-major split below.
    const int S_ = p.tiles_x, K_ = nw / S_;
    const bool grid = K_ >= 2 && (nw - K_ * S_) * 64 <= nw * kGridWaste;
    int ubeg, uend, vband;
    // hybrid split: wave s < S owns rows [0, T_s) of strip s, T_s its weighted share of
    // the pair's units (Tf for the first half of the waves, Tu for the second); the
    // nw - S pool waves march the bottom rows [T_s, H) of all strips, phased (below)
    const bool hyb = !grid && nw > S_ && nw < 2 * S_;
    const int hh = nw >> 1, hsk = nw >= 2 ? p.skew : 0;
    const int hwt = (64 + hsk) * hh + (64 - hsk) * (nw - hh);
    const int hTf = min(H, (U * (64 + hsk)) / hwt), hTu = min(H, (U * (64 - hsk)) / hwt);
    const int hnf = min(hh, S_);
    const bool hpool = hyb && band >= S_;
    // phased pool (round 5): pool wave j marches the bottoms of strips j, j + np, ... (hpFs
    // full rounds; np = nw - S pool waves), so in each phase the pool waves march np adjacent
    // strips side by side and their shared 128-byte lines are fetched about when both need
    // them; then its chunk [hpX0, hpX1) of the remaining strips' bottoms (strip-major from
    // strip hpRb), sized so that each wave's total is its weighted share of the pool units.
    // (The previous strip-major split of the bottoms marched neighbouring strips' shared
    // lines tens of microseconds apart: level-0 reads of a 128-pair launch 1.152x -> 1.135x
    // of the algorithmic bytes, the launch 2061 -> 2052 us, same box.)
    const int hpNp = max(nw - S_, 1), hpJ = band - S_;
    const int hpFs = S_ / hpNp, hpRb = hpFs * hpNp;
    auto hT = [&](int s) { return s < hnf ? hTf : hTu; };
    int hpF = 0, hpX0 = 0, hpX1 = 0;
    if (hpool) {
      int PU = 0, RU = 0;
      for (int s = 0; s < S_; ++s) {
        PU += H - hT(s);
        RU += s >= hpRb ? H - hT(s) : 0;
      }
      int wt = 0;
      for (int i = 0; i < hpNp; ++i) wt += (S_ + i) < hh ? 64 + hsk : 64 - hsk;
      int ws = 0, cf = 0, x = 0;  // running: weight, full-round units, chunk start (a running max)
      for (int i = 0; i <= hpJ; ++i) {
        int fi = 0;
        for (int r = 0; r < hpFs; ++r) fi += H - hT(r * hpNp + i);
        const int wi = (S_ + i) < hh ? 64 + hsk : 64 - hsk;
        const int x1 = i == hpNp - 1 ? RU : max(x, min(max((PU * (ws + wi)) / wt - (cf + fi), 0), RU));
        if (i == hpJ) {
          hpF = fi;
          hpX0 = x;
          hpX1 = x1;
        }
        ws += wi;
        cf += fi;
        x = x1;
      }
    }
    // grid + pool split (2 S < nw, no waste-free grid: the 64-pair launch's 32 waves over 11
    // strips): Kg = ceil(nw / S) row bands with common cuts give Kg S >= nw segments; wave w
    // marches segment w (band w / S, strip w % S) and the Eg = Kg S - nw segments left over
    // (the last band's last strips) are split strip-major over all nw waves, marched after
    // each wave's own segment.  So Eg / (Kg S) of the units (1 in 33 at 64 pairs) run without
    // their horizontal neighbours in lockstep, against all of them on the strip-major split.
    // Band cuts weight each band by its segments' waves (64 + skew in the first half of the
    // pair's waves, 64 - skew in the second, 64 for a left-over segment).
    const int Kg = (nw + S_ - 1) / S_, Eg = Kg * S_ - nw;
    const bool gpool = !grid && !hyb && Kg >= 3;
    auto gp_w = [&](int n) {  // weight of segments 0 .. n - 1
      return (long)(64 + hsk) * min(n, hh) + (long)(64 - hsk) * min(max(n - hh, 0), nw - hh) + 64L * max(n - nw, 0);
    };
    auto gp_cut = [&](int k) { return (int)(((long)H * gp_w(k * S_)) / gp_w(Kg * S_)); };
    const int gk = band / S_, gs = band - gk * S_;
    const int gr0 = gpool ? gp_cut(gk) : 0, gr1 = gpool ? gp_cut(gk + 1) : 0;  // main rows [gr0, gr1)
    const int gL0 = gpool ? gp_cut(Kg - 1) : 0, gHL = H - gL0;                 // the last band's rows
    const int gPU = Eg * gHL, gpb = gpool ? (int)(((long)gPU * band) / nw) : 0;
    const int gpe = gpool ? (int)(((long)gPU * (band + 1)) / nw) : 0;  // pool units [gpb, gpe)
    if (gpool) {
      ubeg = 0;
      uend = (gr1 - gr0) + (gpe - gpb);
      vband = gk;
    } else if (hyb && !hpool) {
      ubeg = band * H;
      uend = band * H + (band < hh ? hTf : hTu);
      vband = 0;
    } else if (hpool) {
      ubeg = 0;
      uend = hpF + hpX1 - hpX0;
      vband = 1;
    } else if (grid) {
      const int k = band / S_, s = band - k * S_;
      ubeg = k < K_ ? s * H + split_start(k, K_, H) : 0;
      uend = k < K_ ? s * H + split_start(k + 1, K_, H) : 0;
      vband = k;
    } else {
      ubeg = split_start(band, nw, U);
      uend = split_start(band + 1, nw, U);
      vband = band;
    }
    const int nrows = uend - ubeg;
    // odd iterations reverse every band: they start on the rows the previous iteration
    // read last, which are still in the Infinity Cache
    const bool up = ((vband & 1) != 0) != (p.reverse != 0);
    const int dir = up ? -1 : 1;
    const float dirf = up ? -1.0f : 1.0f;
    // unit k of the wave's run -> (lane column xs, row y); strt: a strip begins at this
    // row in marching order (row H - 1 marching up, the strip's first row marching down)
    // run: units k, k + 1, ... up to k + run - 1 are rows y, y + dir, ... of the same strip
    auto unit_pos_run = [&](int k, int& xs, int& y, bool& strt, int& run) {
      const int u = up ? uend - 1 - k : ubeg + k;
      int strip, ytop = 0, ylo = 0, yhi = H;  // [ylo, yhi): the rows of this straight run's segment
      if (gpool) {
        const int m = gr1 - gr0;
        if (k < m) {  // own segment (k == 0 primes the window)
          strip = gs;
          y = up ? gr1 - 1 - k : gr0 + k;
          strt = false;
          ylo = gr0;
          yhi = gr1;
        } else {  // pool run: the left-over segments' units gpb .. gpe - 1, strip-major
          const int j = up ? gpe - 1 - (k - m) : gpb + (k - m);
          const int sp = j / gHL;
          strip = S_ - Eg + sp;
          y = gL0 + (j - sp * gHL);
          strt = k == m || y == (up ? H - 1 : gL0);
          ylo = gL0;
        }
      } else {
        if (hpool) {
          // k in marching order: the full rounds' strips first (every pool wave in the same
          // phase), then the chunk; each segment walked in the marching direction
          if (k < hpF) {
            int kk = k, r = 0;
            while (r + 1 < hpFs && kk >= H - hT(r * hpNp + hpJ)) {
              kk -= H - hT(r * hpNp + hpJ);
              ++r;
            }
            strip = r * hpNp + hpJ;
            ylo = hT(strip);
            yhi = H;
            y = up ? H - 1 - kk : ylo + kk;
          } else {
            const int kc = k - hpF;
            const int v = up ? hpX1 - 1 - kc : hpX0 + kc;  // unit of the remaining strips' bottoms
            int s = hpRb, base = 0;
            while (s + 1 < S_ && v >= base + (H - hT(s))) {
              base += H - hT(s);
              ++s;
            }
            strip = s;
            ylo = hT(s) + max(0, hpX0 - base);
            yhi = hT(s) + min(H - hT(s), hpX1 - base);
            y = hT(s) + (v - base);
          }
          strt = y == (up ? yhi - 1 : ylo);
          xs = strip * kTileOut - 1 + lane;
          run = min(up ? y - ylo + 1 : yhi - y, nrows - k);
          return;
        } else {
          strip = u / H;
          y = u - strip * H;
        }
        strt = y == (up ? H - 1 : ytop);
        ylo = ytop;
      }
      xs = strip * kTileOut - 1 + lane;
      run = min(up ? y - ylo + 1 : yhi - y, nrows - k);
    };
    // window in LDS, per wave [2 slots][NQ quads][64 lanes] (each lane only ever touches
    // its own column and a wave's LDS accesses complete in order: no barrier)
    f32x4* win = lds_win[wave];
    float sprev = 0.f, scur = 0.f;
    struct QuadM {
      f32x4 f;      // f0 row y + dir
      f32x4 t[2];   // f1 trailing tap pair (on a tap-cache hit: a re-request of the leading pair)
      f32x4 P;      // minus the partial residual of the cached trailing pair (see issue_t)
    };
    // Tap cache: in marching order, the f1 tap row a pixel row shares with
    // the next one is its LEADING row (lower row marching down, upper row marching up)
    // and the next row's TRAILING row.  Each lane keeps its leading pair of every quad
    // (pair base `tc_ob`) and the next row reloads its trailing pair only where the
    // pair base differs: a hit returns exactly the bytes a load of that base would
    // (f1 is read-only), so the cache changes no result, only the f1 re-fetch that
    // otherwise misses the XCD's L2 one row-step later.
    f32x4 tc[NQW][2];
    int tc_ob = -1;
#pragma unroll
    for (int q = 0; q < NQW; ++q) tc[q][0] = tc[q][1] = f32x4{0.f, 0.f, 0.f, 0.f};  // weighted 0 until cached

    // inverse depth of the next step's pixel, prefetched one step ahead
    float dnx = 0.f;
    auto load_dpx = [&](int xs, int y) { return bld(rd0, y * W * 4 + min(max(xs, 0), W - 1) * 4, 0); };
    constexpr int RM = kRingQ < NQW ? kRingQ : NQW;
    static_assert(RM >= 2 && RM <= NQW && NQW % RM == 0, "ring depth");
    QuadM L[RM];
    // f0 row y + dir of a step's first RM - 1 quads depends on the row only: the previous
    // step issues it into the ring slots its last quads free, so it streams during that
    // step's epilogue and this step's frame (warp, gathers).  (A loop-carried sigma0 row
    // load the same way gets a copy at the loop edge, and the copy waits for every load.)
    // (not with combine_ICP: its per-pixel term leaves no registers for the loop-carried
    // rows -- 256 VGPRs, one wave per SIMD; there the first quads' f0 rows are issued at the
    // start of their own step, before the frame)
    constexpr bool kPf = !ICP;
    auto prefetch_f = [&](int i, int colq, int yn) {
      L[i].f = llvm_buf_load_f32x4(rf0, colq, i * 4 * (int)planeB + yn * W * 16, kF0Aux);
    };
    // the current unit's position, carried from step to step: the next unit is the next row
    // of the same strip while the straight run lasts (cu_run > 1), else (a few times per
    // band) the full unit -> position mapping
    int cu_xs = 0, cu_y = 0, cu_run = 0;
    bool cu_st = false;
    // Normalised coordinates without a division per row: px of the lane's column once per
    // strip (at the window prime), py of 64 rows at a time (lane l: row ny_base + dir l),
    // read back with one v_readlane per row -- the same IEEE divisions, fewer of them
    float nx_lane = 0.f, ny_lanes = 0.f;
    int ny_base = 0;
    auto ny_refresh = [&](int yb) {
      ny_base = yb;
      ny_lanes = norm_coord(min(max(yb + dir * lane, 0), H - 1), cy, fy);
    };
    if (nrows > 0) {
      unit_pos_run(0, cu_xs, cu_y, cu_st, cu_run);
      cu_y = __builtin_amdgcn_readfirstlane(cu_y);
      cu_run = __builtin_amdgcn_readfirstlane(cu_run);
      cu_st = __builtin_amdgcn_readfirstlane((int)cu_st) != 0;
      const int xs0 = cu_xs, y0 = cu_y;
      dnx = load_dpx(xs0, y0);
      ny_refresh(y0);
#pragma unroll
      for (int i = 0; i < RM - 1; ++i)
        if (kPf) prefetch_f(i, min(max(xs0, 0), W - 1) * 16, min(max(y0 + dir, 0), H - 1));
    }
    // One marching step: row y of the wave's strip.  Window slots (LDS): slot 0 = row
    // y - dir, slot 1 = row y; quad q reads both and leaves (y, y + dir) for the next step.
    // The quad loop is straight-line with static quad indices (the tap cache lives in
    // registers), kRingQ quads in flight.
    auto step = [&](int k) {
      const int xs = cu_xs, y = cu_y;
      const bool strt0 = cu_st;
      const float dcur = dnx;
      const int colq = min(max(xs, 0), W - 1) * 16;
      if (k == 0 || strt0) {  // prime the window: rows y - dir (replicate-clamped) and y
        const int yp = min(max(y - dir, 0), H - 1);
        nx_lane = norm_coord(min(max(xs, 0), W - 1), cx, fx);
#pragma unroll
        for (int q = 0; q < NQW; ++q) {
          const int po = q * 4 * (int)planeB;
          win[q * 64 + lane] = llvm_buf_load_f32x4(rf0, colq, po + yp * W * 16, kF0Aux);
          win[(NQW + q) * 64 + lane] = llvm_buf_load_f32x4(rf0, colq, po + y * W * 16, kF0Aux);
        }
        if (CS1 && !NOSIG) {
          sprev = bld(rs0, colq >> 2, yp * W * 4);
          scur = bld(rs0, colq >> 2, y * W * 4);
        }
        // drain here (strip starts only): otherwise the wait counts after the join are the
        // conservative ones of this path, and every row-step waits for its prefetched rows
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      }
      const int yn = min(max(y + dir, 0), H - 1);
      auto issue_f = [&](QuadM& Qm, int q) {
        Qm.f = llvm_buf_load_f32x4(rf0, colq, q * 4 * (int)planeB + yn * W * 16, kF0Aux);
      };
      if (!kPf) {
#pragma unroll
        for (int i = 0; i < RM - 1; ++i) issue_f(L[i], i);
      }
      const float snew = (CS1 && !NOSIG) ? bld(rs0, colq >> 2, yn * W * 4) : 0.f;
      // the next step's (after the last step: this one's again, so that the loads are
      // unconditional -- a load under a branch makes the wait counts of every later quad
      // conservative)
      int xs1, y1, run1;
      bool st1;
      if (cu_run > 1) {
        xs1 = xs;
        y1 = y + dir;
        st1 = false;
        run1 = cu_run - 1;
      } else {
        unit_pos_run(min(k + 1, nrows - 1), xs1, y1, st1, run1);
      }
      // wave-uniform (a loop-carried value the uniformity analysis would otherwise lose)
      cu_xs = xs1;
      cu_y = y1 = __builtin_amdgcn_readfirstlane(y1);
      cu_run = __builtin_amdgcn_readfirstlane(run1);
      cu_st = __builtin_amdgcn_readfirstlane((int)st1) != 0;
      const int colq1 = min(max(xs1, 0), W - 1) * 16, yn1 = min(max(y1 + dir, 0), H - 1);
      // py of this row: lane (y - ny_base) dir of the 64-row block (refreshed past its end or
      // on a jump to another segment)
      const int ny_off = (y - ny_base) * dir;
      if (ny_off < 0 || ny_off >= 64) ny_refresh(y);
      const float xyr[2] = {nx_lane, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ny_lanes), (y - ny_base) * dir))};
      Frame F;
      {
        const float dv[1] = {dcur};
        make_frame_xy(xs, y, dv, F, false, xyr);
      }
      // after the frame has consumed dcur: the new load then reuses its registers (a
      // loop-carried copy of a register with a load in flight would wait for every load)
      dnx = load_dpx(xs1, y1);  // unconditional (clamped to the last row): no phi of the old value
      // tap cache: trailing / leading pair bases and weights of this row
      const int obT = up ? F.tp[0].ob1 : F.tp[0].ob0, obL = up ? F.tp[0].ob0 : F.tp[0].ob1;
      const bool tc_hit = obT == tc_ob;
      PairWeights wq;  // channel-unit weights of slots t[0..3]
      tc_ob = obL;
      // slots 0/1 hold the trailing pair: the lower row when marching up
      wq.w0 = sel_uniform(up, F.pw[0].w2, F.pw[0].w0);
      wq.w1 = sel_uniform(up, F.pw[0].w3, F.pw[0].w1);
      wq.w2 = sel_uniform(up, F.pw[0].w0, F.pw[0].w2);
      wq.w3 = sel_uniform(up, F.pw[0].w1, F.pw[0].w3);
      // Tap weights split by the cache: on a hit the cached trailing pair carries the
      // trailing weights (w0h, w1h) and the loaded one 0; on a miss the other way round.
      const float w0h = tc_hit ? wq.w0 : 0.f, w1h = tc_hit ? wq.w1 : 0.f;
      const float w0m = tc_hit ? 0.f : wq.w0, w1m = tc_hit ? 0.f : wq.w1;
      auto issue_t = [&](QuadM& Qm, int q) {
        const int po = q * 4 * (int)planeB;
        // The cached trailing pair of quad q is consumed here, before the new leading pair
        // is loaded into its registers (no copy of the cache per row):
        // P = w1h tc1 + (w0h tc0 - fm), fm = f0 row y from the window -- the first two terms
        // of the residual, in the order the residual sums them (below).  On a miss P = -fm.
        // (stored negated, -P = fm - w0h tc0 - w1h tc1 exactly: the negation then folds into the
        // consuming fma as a source modifier instead of a v_xor per element)
        const f32x4 fm = win[(NQW + q) * 64 + lane];
        Qm.P = __builtin_elementwise_fma(f32x4{-w1h, -w1h, -w1h, -w1h}, tc[q][1],
                                         __builtin_elementwise_fma(f32x4{-w0h, -w0h, -w0h, -w0h}, tc[q][0], fm));
        // branch-free: a hit lane re-requests its leading pair (an L1 hit next to the
        // leading loads below), weighted 0; a divergent branch around the loads would make
        // the waitcnt bookkeeping wait on the next quad's loads
        const int offT = (tc_hit ? obL : obT) * 16;
        Qm.t[0] = bld4(rf1, offT, po);
        Qm.t[1] = bld4(rf1, offT + 16, po);
        tc[q][0] = bld4(rf1, obL * 16, po);  // the leading pair: this row's, and the next row's cache
        tc[q][1] = bld4(rf1, obL * 16 + 16, po);
      };
#pragma unroll
      for (int i = 0; i < RM - 1; ++i) issue_t(L[i], i);
      f32x2 Q[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) Q[i] = f32x2{0.f, 0.f};
      auto unitc = [&](int q, const QuadM& cur) {
        f32x4* s0p = win + q * 64 + lane;          // slot 0
        f32x4* s1p = win + (NQW + q) * 64 + lane;  // slot 1
        const f32x4 wtop = *s0p, wmid = *s1p;      // rows above / at the pixel in marching order
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // channels 4q + 2h, 4q + 2h + 1
          auto half = [&](const f32x4& v) { return h ? f32x2{v.z, v.w} : f32x2{v.x, v.y}; };
          const f32x2 fp = half(wtop), fm = half(wmid), fn = half(cur.f);
          const f32x2 V = (fp + fn) + 2.0f * fm;
          // D in marching order: gy carries the sign dirf, folded into the odd sums
          // (gx gy, gy res, gy) once per row below
          const f32x2 D = fn - fp;
          // scalar lane differences: one of each pair of lane shifts folds into the
          // v_sub / v_add as its DPP operand (a packed v_pk_add cannot take one)
          const float xl0 = lane_from_left(V.x), xl1 = lane_from_left(V.y);
          const float dl0 = lane_from_left(D.x), dl1 = lane_from_left(D.y);
          float x0 = lane_from_right(V.x) - xl0, x1 = lane_from_right(V.y) - xl1;
          float y0 = lane_from_right(D.x) + dl0, y1 = lane_from_right(D.y) + dl1;
          // opaque to the SLP vectorizer, which would pack each pair into one v_pk_add
          // and keep both shifts as v_mov_dpp
          asm("" : "+v"(x0), "+v"(x1), "+v"(y0), "+v"(y1));
          const f32x2 x = f32x2{x0, x1};
          const f32x2 yv = f32x2{y0, y1} + 2.0f * D;
          const f32x2 n2 = x * x + (yv * yv + 1e-8f);
          const f32x2 inv = f32x2{__builtin_amdgcn_rsqf(n2.x), __builtin_amdgcn_rsqf(n2.y)};
          const f32x2 gx = x * inv, gy = yv * inv;
          // ((T0 w0 - fm) + T1 w1) + t2 w2 + t3 w3 with T the trailing pair (cached on a hit):
          // the hit and miss halves of each trailing term are exact (one factor is 0), so the
          // sum is the one a select of T would give, bit for bit
          const f32x2 rt = __builtin_elementwise_fma(f32x2{w1m, w1m}, half(cur.t[1]),
                                                     __builtin_elementwise_fma(f32x2{w0m, w0m}, half(cur.t[0]), -half(cur.P)));
          const f32x2 res = __builtin_elementwise_fma(f32x2{wq.w3, wq.w3}, half(tc[q][1]),
                                                      __builtin_elementwise_fma(f32x2{wq.w2, wq.w2}, half(tc[q][0]), rt));
          Q[0] += gx * gx;
          Q[1] += gx * gy;
          Q[2] += gy * gy;
          Q[3] += gx * res;
          Q[4] += gy * res;
          Q[5] += res * res;
          Q[6] += gx;
          Q[7] += gy;
          Q[8] += res;
        }
        // straight-line code: the accumulators are pure arithmetic, which the DAG scheduler
        // would otherwise sink below every later load (all quads' loads first: 400 VGPRs)
        asm volatile("" : "+v"(Q[0]), "+v"(Q[1]), "+v"(Q[2]), "+v"(Q[3]), "+v"(Q[4]), "+v"(Q[5]), "+v"(Q[6]),
                     "+v"(Q[7]), "+v"(Q[8])::"memory");
        *s0p = wmid;  // window (y, y + dir)
        *s1p = cur.f;
      };
      // each unit's accumulators are pinned at its end (unitc), so the rounds keep this order
#pragma unroll
      for (int qq = 0; qq < NQW; ++qq) {
        if (qq + RM - 1 < NQW) {
          issue_f(L[(qq + RM - 1) % RM], qq + RM - 1);
          issue_t(L[(qq + RM - 1) % RM], qq + RM - 1);
        } else if (kPf) {  // the next step's quad qq + RM - 1 - NQW into the freed slot
          prefetch_f(qq + RM - 1 - NQW, colq1, yn1);
        }
        unitc(qq, L[qq % RM]);
      }
      // combine_ICP: the pixel's depth0, loaded here (after the channel loop: no register
      // across it) so that the sigma / pixel terms below run while it loads
      const float d0e = ICP ? p.depth0[(size_t)b * HW + y * W + min(max(xs, 0), W - 1)] : 0.f;
      // the frame's gathers and the sigma0 row are resolved after the channel loop (a
      // select of a loaded value under the wave-uniform direction becomes a branch whose
      // copies wait for every load in flight, before the first tap is issued)
      if (CS1 && !NOSIG) {
        // sigma0 rows top / centre / bottom (marching direction folded in)
        F.s0r[0] = sel_uniform(up, snew, sprev);
        F.s0r[1] = scur;
        F.s0r[2] = sel_uniform(up, sprev, snew);
        sprev = scur;
        scur = snew;
      }
      PixelTerms T;
      pixel_terms(F, T);
      Sums S;
      float q[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) q[i] = Q[i].x + Q[i].y;
      q[1] *= dirf;  // gy was accumulated in marching order
      q[4] *= dirf;
      q[7] *= dirf;
      const float A = T.inv_s[0], bx = T.kk[0] * T.hx[0], by = T.kk[0] * T.hy[0], A2 = A * A;
      S.Saa[0] = A2 * q[0] + 2.0f * A * bx * q[3] + bx * bx * q[5];
      S.Sab[0] = A2 * q[1] + A * by * q[3] + A * bx * q[4] + bx * by * q[5];
      S.Sbb[0] = A2 * q[2] + 2.0f * A * by * q[4] + by * by * q[5];
      S.Sa[0] = A * q[6] + bx * q[8];
      S.Sb[0] = A * q[7] + by * q[8];
      S.Sar[0] = A2 * q[3] + A * bx * q[5];
      S.Sbr[0] = A2 * q[4] + A * by * q[5];
      finish_pixels(F, T, S, &d0e);
    };
    for (int k = 0; k < nrows; ++k) step(k);
  } else if constexpr (C4) {
    // ---- channel-quad layout: the per-pixel weights factor out of the channel sums
    // (alpha = 1/sigma, bx = kk hx, by = kk hy give na = alpha gx + bx r,
    // nb = alpha gy + by r, rw = alpha r for every channel), so the channel loop needs
    // only the taps: nine weight-free sums per pixel,
    // Q = [gx gx, gx gy, gy gy, gx r, gy r, r r, gx, gy, r], accumulated per channel
    // pair in packed fp32 (even / odd channels in the two halves).
    // Quad plane q of pair b = [H][W][4] floats at b * C * HW + q * 4 * HW.
    // (Issuing the next tile's first quads during this tile -- software pipelining
    // across tiles -- needs two live frames: 300 VGPRs, one wave per SIMD, 30 % slower.)
    QuadLoadsR<R> S4[kRing];
    auto issue4 = [&](const Frame& F, QuadLoadsR<R>& L, int k) {
      const int po = k * 4 * (int)planeB;
#pragma unroll
      for (int j = 0; j < R + 2; ++j) L.f[j] = bld4(rf0, F.colv * 4, po + F.rows[j] * 4);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        L.t[r][0] = bld4(rf1, F.tp[r].ob0 * 16, po);
        L.t[r][1] = bld4(rf1, F.tp[r].ob0 * 16 + 16, po);
        L.t[r][2] = bld4(rf1, F.tp[r].ob1 * 16, po);
        L.t[r][3] = bld4(rf1, F.tp[r].ob1 * 16 + 16, po);
      }
    };
    float d_cur[R];
    load_d(seg_begin, d_cur);
    for (int it = seg_begin; it < seg_end; ++it) {
      float dv[R];
#pragma unroll
      for (int r = 0; r < R; ++r) dv[r] = d_cur[r];
      if (it + 1 < seg_end) load_d(it + 1, d_cur);
      Frame F;
      make_frame(it, dv, F);
      if (F.skip) continue;
#pragma unroll
      for (int q = 0; q + 1 < kRing; ++q)
        if (q < nch) issue4(F, S4[q], q);
      // resolve the frame's gathers now (issued before the quads: no wait on those), so
      // that only the taps, weights and epilogue inputs stay live across the channel loop
      PixelTerms T;
      pixel_terms(F, T);
      {
        f32x2 Q[R][9];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
          for (int k = 0; k < 9; ++k) Q[r][k] = f32x2{0.f, 0.f};
        // two channels of row r (lane-neighbour terms by DPP per half)
        auto chan2 = [&](int r, f32x2 ft, f32x2 fm, f32x2 fb, f32x2 t0, f32x2 t1, f32x2 t2, f32x2 t3) {
          const f32x2 V = ft + 2.0f * fm + fb;
          const f32x2 D = fb - ft;
          const f32x2 x = f32x2{lane_from_right(V.x) - lane_from_left(V.x), lane_from_right(V.y) - lane_from_left(V.y)};
          const f32x2 y =
              f32x2{lane_from_left(D.x) + lane_from_right(D.x), lane_from_left(D.y) + lane_from_right(D.y)} + 2.0f * D;
          const f32x2 n2 = x * x + y * y + 1e-8f;
          const f32x2 inv = f32x2{__builtin_amdgcn_rsqf(n2.x), __builtin_amdgcn_rsqf(n2.y)};
          const f32x2 gx = x * inv, gy = y * inv;
          const PairWeights& w = F.pw[r];
          const f32x2 res = (t0 * w.w0 + t1 * w.w1 + t2 * w.w2 + t3 * w.w3) - fm;
          Q[r][0] += gx * gx;
          Q[r][1] += gx * gy;
          Q[r][2] += gy * gy;
          Q[r][3] += gx * res;
          Q[r][4] += gy * res;
          Q[r][5] += res * res;
          Q[r][6] += gx;
          Q[r][7] += gy;
          Q[r][8] += res;
        };
        auto unit = [&](int k, QuadLoadsR<R>& cur, QuadLoadsR<R>& nxt, bool refill) {
          if (refill && k + kRing - 1 < nch) issue4(F, nxt, k + kRing - 1);
          if (k >= nch) return;
#pragma unroll
          for (int h = 0; h < 2; ++h) {  // channels 4k + 2h, 4k + 2h + 1
#pragma unroll
            for (int r = 0; r < R; ++r) {
              auto half = [&](const f32x4& v) { return h ? f32x2{v.z, v.w} : f32x2{v.x, v.y}; };
              chan2(r, half(cur.f[r]), half(cur.f[r + 1]), half(cur.f[r + 2]), half(cur.t[r][0]),
                    half(cur.t[r][1]), half(cur.t[r][2]), half(cur.t[r][3]));
            }
          }
        };
        // every group but the last refills the ring unconditionally (no register merges in the loop)
#pragma unroll 1
        for (int kq = 0; kq < nunits - kRing; kq += kRing) {
#pragma unroll
          for (int q = 0; q < kRing; ++q) unit(kq + q, S4[q], S4[(q + kRing - 1) % kRing], true);
        }
#pragma unroll
        for (int q = 0; q < kRing; ++q) unit(nunits - kRing + q, S4[q], S4[(q + kRing - 1) % kRing], q == 0);

        Sums S;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          float q[9];
#pragma unroll
          for (int k = 0; k < 9; ++k) q[k] = Q[r][k].x + Q[r][k].y;
          const float A = T.inv_s[r], bx = T.kk[r] * T.hx[r], by = T.kk[r] * T.hy[r], A2 = A * A;
          S.Saa[r] = A2 * q[0] + 2.0f * A * bx * q[3] + bx * bx * q[5];
          S.Sab[r] = A2 * q[1] + A * by * q[3] + A * bx * q[4] + bx * by * q[5];
          S.Sbb[r] = A2 * q[2] + 2.0f * A * by * q[4] + by * by * q[5];
          S.Sa[r] = A * q[6] + bx * q[8];
          S.Sb[r] = A * q[7] + by * q[8];
          S.Sar[r] = A2 * q[3] + A * bx * q[5];
          S.Sbr[r] = A2 * q[4] + A * by * q[5];
        }
        finish_pixels(F, T, S);
      }
    }
  } else {
    // ---- NCHW layout: per channel, three f0 rows and two tap pairs per pixel
    float d_cur[R];
    load_d(seg_begin, d_cur);
    for (int it = seg_begin; it < seg_end; ++it) {
      float dv[R];
#pragma unroll
      for (int r = 0; r < R; ++r) dv[r] = d_cur[r];
      if (it + 1 < seg_end) load_d(it + 1, d_cur);
      Frame F;
      make_frame(it, dv, F);
      if (F.skip) continue;
      const int colv = F.colv;
      ChanLoadsR<R> S[kRing][kCK];
      auto issue = [&](ChanLoadsR<R> (&L)[kCK], int k) {
#pragma unroll
        for (int cc = 0; cc < kCK; ++cc) {
          const int c = k * kCK + cc;
          if (c < C) {
            const int po = c * (int)planeB;
#pragma unroll
            for (int j = 0; j < R + 2; ++j) L[cc].f[j] = bld(rf0, colv, po + F.rows[j]);
#pragma unroll
            for (int r = 0; r < R; ++r) L[cc].g[r] = gather4(rf1, F.tp[r], po);
          }
        }
      };
#pragma unroll
      for (int q = 0; q + 1 < kRing; ++q) issue(S[q], q);
      PixelTerms T;
      pixel_terms(F, T);
      Sums Sm;
#pragma unroll
      for (int r = 0; r < R; ++r) Sm.Saa[r] = Sm.Sab[r] = Sm.Sbb[r] = Sm.Sa[r] = Sm.Sb[r] = Sm.Sar[r] = Sm.Sbr[r] = 0.f;

      // one channel of row r: ft, fm, fb = f0 column above / at / below the pixel, g = f1 taps
      auto chan = [&](int r, int c, float ft, float fm, float fb, const Gather4& g) {
        float gx, gy;
        sobel_cols(ft, fm, fb, gx, gy);
        float is_c = T.inv_s[r], kk_c = T.kk[r], hx_c = T.hx[r], hy_c = T.hy[r];
        if (!CS1 && !NOSIG) {  // per-channel sigma (R == 1 here)
          const int po = c * (int)planeB;
          const float st_ = bld(rs0, colv, po + F.rows[0]), sm_ = bld(rs0, colv, po + F.rows[1]),
                      sb_ = bld(rs0, colv, po + F.rows[2]);
          sobel_cols(st_, sm_, sb_, hx_c, hy_c);
          const float src = bil(p.s1 + ((size_t)b * p.Cs + c) * HW, F.tp[r]);
          const float sg = sqrtf(src * src + sm_ * sm_);
          is_c = 1.0f / sg;
          kk_c = sm_ * (is_c * is_c * is_c);
          if (c == 0) {
            T.sr0[r] = src;
            T.srmin[r] = T.srmax[r] = src;
            if (TRU) T.invalid[r] = T.invalid[r] || (sm_ == g0min) || (sm_ == g0max);
          } else {
            T.srmin[r] = fminf(T.srmin[r], src);
            T.srmax[r] = fmaxf(T.srmax[r], src);
          }
        }
        const float frv = bilp(g, F.pw[r]);
        const float res = frv - fm;
        const float rw = res * is_c;
        const float rk = res * kk_c;
        // na = -a, nb = -b (a, b of algorithms.py:872); the linear sums are negated in finish_pixels
        const float na = gx * is_c + rk * hx_c;
        const float nb = gy * is_c + rk * hy_c;
        Sm.Saa[r] += na * na;
        Sm.Sab[r] += na * nb;
        Sm.Sbb[r] += nb * nb;
        Sm.Sa[r] += na;
        Sm.Sb[r] += nb;
        Sm.Sar[r] += na * rw;
        Sm.Sbr[r] += nb * rw;
      };
      auto unit = [&](int k, ChanLoadsR<R> (&cur)[kCK], ChanLoadsR<R> (&nxt)[kCK], bool refill) {
        if (refill) issue(nxt, k + kRing - 1);
#pragma unroll
        for (int cc = 0; cc < kCK; ++cc) {
          const int c = k * kCK + cc;
          if (c >= C) break;
#pragma unroll
          for (int r = 0; r < R; ++r) chan(r, c, cur[cc].f[r], cur[cc].f[r + 1], cur[cc].f[r + 2], cur[cc].g[r]);
        }
      };
      // every group but the last refills the ring unconditionally (no register merges in the loop)
#pragma unroll 1
      for (int kq = 0; kq < nunits - kRing; kq += kRing) {
#pragma unroll
        for (int q = 0; q < kRing; ++q) unit(kq + q, S[q], S[(q + kRing - 1) % kRing], true);
      }
#pragma unroll
      for (int q = 0; q < kRing; ++q) unit(nunits - kRing + q, S[q], S[(q + kRing - 1) % kRing], q == 0);
      finish_pixels(F, T, Sm);
    }
  }

  // ---- workgroup reduction -> one record (fixed order: deterministic)
#pragma unroll
  for (int k = 0; k < 27; ++k) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc[k] += __shfl_xor(acc[k], off);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ninv += __shfl_xor(ninv, off);
  Extremum emn, emx;
  if (TRU) {
    emn.all = mn_all;
    emn.v0 = mn0;
    emx.all = mx_all;
    emx.v0 = mx0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      emn.c[k] = lds_ext[k][tid];
      emx.c[k] = lds_ext[7 + k][tid];
    }
    emn.n = lds_ext[6][tid];
    emx.n = lds_ext[13][tid];
    ext_wave_reduce<true>(emn);
    ext_wave_reduce<false>(emx);
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 27; ++k) red[wave][k] = acc[k];
    red[wave][R_NINV] = ninv;
    if (TRU) {
      red[wave][R_MN_ALL] = emn.all;
      red[wave][R_MN0] = emn.v0;
      red[wave][R_NMN] = emn.n;
      red[wave][R_MX_ALL] = emx.all;
      red[wave][R_MX0] = emx.v0;
      red[wave][R_NMX] = emx.n;
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        red[wave][R_CMN + k] = emn.c[k];
        red[wave][R_CMX + k] = emx.c[k];
      }
    }
  }
  __syncthreads();
  float* out = p.rec + (size_t)kb * kRec;
  if (tid < 28) {
    st_ag(out + tid, (float)(((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid]));
  } else if (TRU && tid == 64) {
    Extremum e;
    e.all = red[0][R_MN_ALL];
    e.v0 = red[0][R_MN0];
    e.n = red[0][R_NMN];
    for (int k = 0; k < 6; ++k) e.c[k] = red[0][R_CMN + k];
    for (int w = 1; w < 4; ++w) ext_merge<true>(e, red[w][R_MN_ALL], red[w][R_MN0], &red[w][R_CMN], red[w][R_NMN]);
    st_ag(out + R_MN_ALL, (float)(e.all));
    st_ag(out + R_MN0, (float)(e.v0));
    st_ag(out + R_NMN, (float)(e.n));
    for (int k = 0; k < 6; ++k) st_ag(out + R_CMN + k, (float)(e.c[k]));
  } else if (TRU && tid == 128) {
    Extremum e;
    e.all = red[0][R_MX_ALL];
    e.v0 = red[0][R_MX0];
    e.n = red[0][R_NMX];
    for (int k = 0; k < 6; ++k) e.c[k] = red[0][R_CMX + k];
    for (int w = 1; w < 4; ++w) ext_merge<false>(e, red[w][R_MX_ALL], red[w][R_MX0], &red[w][R_CMX], red[w][R_NMX]);
    st_ag(out + R_MX_ALL, (float)(e.all));
    st_ag(out + R_MX0, (float)(e.v0));
    st_ag(out + R_NMX, (float)(e.n));
    for (int k = 0; k < 6; ++k) st_ag(out + R_CMX + k, (float)(e.c[k]));
  }
  // the last workgroup of a pair reduces its records; the one completing the batch solves
  // the batch-last workgroup reduces every pair's records and solves (LDS scratch: the
  // marching window, else the extremum buffer -- both dead by now)
  if (p.fin_on && block_is_last(p.fin.pair_cnt + b, 1u, (uint32_t)p.nbpp)) {
    if constexpr (kWin)
      pair_reduce2(p.fin, b, reinterpret_cast<float*>(&lds_win[0][0]));
    else if constexpr (TRU)
      pair_reduce2(p.fin, b, &lds_ext[0][0]);
    else
      pair_reduce2(p.fin, b, fin_sc);
    finalize_group(p.fin, b);
  }
}

// ============================================================ split normal-equation accumulation
// Kernels whose 4 waves cooperate on the same pixels (each wave a share of the channel
// quads) meet in LDS with the per-pixel channel sums; then every wave accumulates a
// quarter of the 27 normal-equation entries of the same pixels: wave w < 3 the JtJ
// upper-triangle entries 7w .. 7w + 6 (row-major), wave 3 the six JtR entries, the
// invalid count and the truncated-sigma extremum bookkeeping (finish_pixels' logic).
template <bool TRU, bool NOSIG, int NW = 4>
struct SplitAcc {
  static constexpr float kFill = NOSIG ? 1e-3f : 1e-6f;  // weighted residual of invalid pixels
  static constexpr int EPW = (21 + NW - 2) / (NW - 1);   // JtJ entries per wave (waves 0 .. NW-2)
  static constexpr int NA = EPW > 7 ? EPW : 7;           // the last wave: 6 JtR + invalid count
  float accw[NA];
  float mn_all, mn0, mx_all, mx0;

  __device__ __forceinline__ void init(int wave, int lane, float (*lds_ext)[64]) {
#pragma unroll
    for (int i = 0; i < NA; ++i) accw[i] = 0.0f;
    mn_all = mn0 = INFINITY;
    mx_all = mx0 = -INFINITY;
    if (TRU && wave == NW - 1) {
#pragma unroll
      for (int i = 0; i < 14; ++i) lds_ext[i][lane] = 0.0f;
    }
  }

  // Sa, Sb, Sar, Sbr already negated (the linear terms of J_c = -(a_c Jx + b_c Jy))
  template <int w>
  __device__ __forceinline__ void add_w(int lane, float Saa, float Sab, float Sbb, float Sa, float Sb, float Sar,
                                        float Sbr, const float* Jx, const float* Jy, bool invalid, float sr,
                                        float (*lds_ext)[64]) {
    if constexpr (w < NW - 1) {
      int kq = 0;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const float Pi = Saa * Jx[i] + Sab * Jy[i], Qi = Sab * Jx[i] + Sbb * Jy[i];
#pragma unroll
        for (int j = i; j < 6; ++j) {
          if (kq >= EPW * w && kq < EPW * w + EPW) accw[kq - EPW * w] += Pi * Jx[j] + Qi * Jy[j];
          ++kq;
        }
      }
    } else {
      const float cA = invalid ? kFill * Sa : Sar;
      const float cB = invalid ? kFill * Sb : Sbr;
#pragma unroll
      for (int i = 0; i < 6; ++i) accw[i] -= cA * Jx[i] + cB * Jy[i];
      accw[6] += invalid ? 1.0f : 0.0f;
      if (TRU) {
        mn_all = fminf(mn_all, sr);
        mx_all = fmaxf(mx_all, sr);
        const bool le = sr <= mn0, ge = sr >= mx0;
        if (le || ge) {
          float corr[7];
          const float dA = invalid ? 0.0f : (1e-6f * Sa - Sar);
          const float dB = invalid ? 0.0f : (1e-6f * Sb - Sbr);
#pragma unroll
          for (int i = 0; i < 6; ++i) corr[i] = -(dA * Jx[i] + dB * Jy[i]);
          corr[6] = invalid ? 0.0f : 1.0f;
          if (le) {
            const bool reset = sr < mn0;
            mn0 = sr;
#pragma unroll
            for (int i = 0; i < 7; ++i) lds_ext[i][lane] = (reset ? 0.0f : lds_ext[i][lane]) + corr[i];
          }
          if (ge) {
            const bool reset = sr > mx0;
            mx0 = sr;
#pragma unroll
            for (int i = 0; i < 7; ++i) lds_ext[7 + i][lane] = (reset ? 0.0f : lds_ext[7 + i][lane]) + corr[i];
          }
        }
      }
    }
  }
  template <int w = 0>
  __device__ __forceinline__ void add(int wave, int lane, float Saa, float Sab, float Sbb, float Sa, float Sb,
                                      float Sar, float Sbr, const float* Jx, const float* Jy, bool invalid, float sr,
                                      float (*lds_ext)[64]) {
    if (wave == w || w == NW - 1) {
      add_w<w>(lane, Saa, Sab, Sbb, Sa, Sb, Sar, Sbr, Jx, Jy, invalid, sr, lds_ext);
    } else if constexpr (w + 1 < NW) {
      add<w + 1>(wave, lane, Saa, Sab, Sbb, Sa, Sb, Sar, Sbr, Jx, Jy, invalid, sr, lds_ext);
    }
  }

  // Workgroup record: wave w < NW-1 holds JtJ entries EPW w .. EPW w + EPW - 1, the last
  // wave JtR, the invalid count and the truncated-sigma extrema.
  __device__ __forceinline__ void write_record(int wave, int lane, float (*lds_ext)[64], float* red, float* out) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) accw[i] += __shfl_xor(accw[i], off);
    }
    if (lane == 0) {
      if (wave < NW - 1) {
#pragma unroll
        for (int i = 0; i < EPW; ++i)
          if (EPW * wave + i < 21) red[EPW * wave + i] = accw[i];
      } else {
#pragma unroll
        for (int i = 0; i < 7; ++i) red[21 + i] = accw[i];
      }
    }
    if (TRU && wave == NW - 1) {
      Extremum emn, emx;
      emn.all = mn_all;
      emn.v0 = mn0;
      emx.all = mx_all;
      emx.v0 = mx0;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        emn.c[i] = lds_ext[i][lane];
        emx.c[i] = lds_ext[7 + i][lane];
      }
      emn.n = lds_ext[6][lane];
      emx.n = lds_ext[13][lane];
      ext_wave_reduce<true>(emn);
      ext_wave_reduce<false>(emx);
      if (lane == 0) {
        red[R_MN_ALL] = emn.all;
        red[R_MN0] = emn.v0;
        red[R_NMN] = emn.n;
        red[R_MX_ALL] = emx.all;
        red[R_MX0] = emx.v0;
        red[R_NMX] = emx.n;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          red[R_CMN + i] = emn.c[i];
          red[R_CMX + i] = emx.c[i];
        }
      }
    }
    __syncthreads();
    const int tid = threadIdx.x;
    if (tid < (TRU ? R_NMX + 1 : R_NINV + 1)) st_ag(out + tid, red[tid]);
  }
};

// Stand-alone finalize (one workgroup per pair): pair records, then the batch solve.
__global__ __launch_bounds__(kThreads) void finalize_kernel(FinParams q) {
  __shared__ float sc[kFinScratch];
  pair_reduce2(q, blockIdx.x, sc);
  finalize_group(q, blockIdx.x);
}

// ============================================================ channel-split reduce kernel (coarse levels)
// Channel-quad layout, one sigma plane, U_IC (MODE 0) or IC (MODE 2), C % 16 == 0.
// For the small pyramid levels, where a wave that walks all channels of a row is a
// chain of ~10 dependent memory latencies and the device is far from full: one
// workgroup per (column strip, row) unit (grid-stride over a pair's units), its 4
// waves split the channel quads, and every wave issues ALL of its loads for the unit
// at once (f0 rows y-1, y, y+1 and the f1 taps of each of its quads).  The warp /
// taps / sigma terms are recomputed by each wave (cheap next to the latency they
// save); the per-pixel channel sums meet in LDS behind one barrier per unit and
// each wave accumulates its share of the normal equations (SplitAcc).
// One pass of the channel-split schedule over pair b's units jb, jb + stride, ...:
// the workgroup's record goes to `out`.
template <int CT, bool TRU, int MODE>
__device__ __forceinline__ void split_pass(const IterParams& p, int b, int jb, int stride, float (&qs)[2][4][9][64],
                                           float (*lds_ext)[64], float* red, float* out) {
  constexpr bool NOSIG = MODE == 2;
  constexpr int NQ = CT / 4, QW = NQ / 4;
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int W = p.W, H = p.H, HW = H * W;
  const int U = p.tiles_x * H;
  const int grp2 = 2 * (b / p.fin.group);  // this pair's batch: its sigma0 extrema
  const float g0min = TRU ? dec_ord(p.ext[grp2]) : 0.f, g0max = TRU ? dec_ord(p.ext[grp2 + 1]) : 0.f;
  const uint32_t planeB = (uint32_t)HW * 4u;
  const float fx = p.K[4 * b + 0], fy = p.K[4 * b + 1], cx = p.K[4 * b + 2], cy = p.K[4 * b + 3];
  float Rm[9], tv[3];
#pragma unroll
  for (int k = 0; k < 9; ++k) Rm[k] = p.R[9 * b + k];
#pragma unroll
  for (int k = 0; k < 3; ++k) tv[k] = p.t[3 * b + k];
  const auto rf0 = rsrc(p.f0 + (size_t)b * CT * HW, planeB * CT);
  const auto rf1 = rsrc(p.f1 + (size_t)b * CT * HW, planeB * CT);
  const auto rs0 = rsrc(NOSIG ? p.invD0 : p.s0 + (size_t)b * HW, planeB);
  const auto rs1 = rsrc(NOSIG ? p.invD0 : p.s1 + (size_t)b * HW, planeB);
  const auto rd0 = rsrc(p.invD0 + (size_t)b * HW, planeB);
  const auto rd1 = rsrc(p.invD1 + (size_t)b * HW, planeB);
  const uint8_t* m0b = p.mask0 ? p.mask0 + (size_t)b * HW : nullptr;
  const uint8_t* m1b = p.mask1 ? p.mask1 + (size_t)b * HW : nullptr;

  SplitAcc<TRU, NOSIG> acc;
  acc.init(wave, lane, lds_ext);

  auto unit_xy = [&](int u, int& xc, int& y, bool& out_lane) {
    const int strip = u / H;
    y = u - strip * H;
    const int xs = strip * kTileOut - 1 + lane;
    xc = min(max(xs, 0), W - 1);
    out_lane = (lane >= 1) && (lane <= kTileOut) && (xs < W);
  };
  float dnext = 0.f;
  if (jb < U) {
    int xc, y;
    bool ol;
    unit_xy(jb, xc, y, ol);
    dnext = bld(rd0, y * W * 4 + xc * 4, 0);
  }
  int par = 0;
  for (int u = jb; u < U; u += stride, par ^= 1) {
    int xc, y;
    bool out_lane;
    unit_xy(u, xc, y, out_lane);
    const float d = dnext;
    if (u + stride < U) {
      int xn, yn;
      bool oln;
      unit_xy(u + stride, xn, yn, oln);
      dnext = bld(rd0, yn * W * 4 + xn * 4, 0);
    }
    const Warp fw = warp_point(xc, y, d, Rm, tv, fx, fy, cx, cy);
    const Taps tp = make_taps(fw.u, fw.v, H, W);
    const PairWeights pw = pair_weights(tp);
    const Gather4 gd1 = gather4(rd1, tp, 0);
    Gather4 gs1{0.f, 0.f, 0.f, 0.f};
    float s0t = 0.f, s0m = 0.f, s0b = 0.f;
    const int yt = max(y - 1, 0), yb = min(y + 1, H - 1);
    if (!NOSIG) {
      gs1 = gather4(rs1, tp, 0);
      s0t = bld(rs0, xc * 4, yt * W * 4);
      s0m = bld(rs0, xc * 4, y * W * 4);
      s0b = bld(rs0, xc * 4, yb * W * 4);
    }
    f32x4 ft[QW], fm[QW], fb[QW], t[QW][4];
#pragma unroll
    for (int qq = 0; qq < QW; ++qq) {
      const int po = (wave * QW + qq) * 4 * (int)planeB;
      ft[qq] = bld4(rf0, xc * 16, po + yt * W * 16);
      fm[qq] = bld4(rf0, xc * 16, po + y * W * 16);
      fb[qq] = bld4(rf0, xc * 16, po + yb * W * 16);
      t[qq][0] = bld4(rf1, tp.ob0 * 16, po);
      t[qq][1] = bld4(rf1, tp.ob0 * 16 + 16, po);
      t[qq][2] = bld4(rf1, tp.ob1 * 16, po);
      t[qq][3] = bld4(rf1, tp.ob1 * 16 + 16, po);
    }
    const bool fm0 = m0b ? (m0b[y * W + xc] != 0) : true;
    const float fm1 = m1b ? bil_u8(m1b, tp) : 1.0f;
    // channel sums of this wave's quads
    f32x2 Q[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) Q[i] = f32x2{0.f, 0.f};
#pragma unroll
    for (int qq = 0; qq < QW; ++qq) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        auto half = [&](const f32x4& v) { return h ? f32x2{v.z, v.w} : f32x2{v.x, v.y}; };
        const f32x2 a = half(ft[qq]), c = half(fm[qq]), e = half(fb[qq]);
        const f32x2 V = (a + e) + 2.0f * c;
        const f32x2 D = e - a;
        const f32x2 x = f32x2{lane_from_right(V.x) - lane_from_left(V.x), lane_from_right(V.y) - lane_from_left(V.y)};
        const f32x2 yv =
            f32x2{lane_from_left(D.x) + lane_from_right(D.x), lane_from_left(D.y) + lane_from_right(D.y)} + 2.0f * D;
        const f32x2 n2 = x * x + yv * yv + 1e-8f;
        const f32x2 inv = f32x2{__builtin_amdgcn_rsqf(n2.x), __builtin_amdgcn_rsqf(n2.y)};
        const f32x2 gx = x * inv, gy = yv * inv;
        const f32x2 res =
            (half(t[qq][0]) * pw.w0 + half(t[qq][1]) * pw.w1 + half(t[qq][2]) * pw.w2 + half(t[qq][3]) * pw.w3) - c;
        Q[0] += gx * gx;
        Q[1] += gx * gy;
        Q[2] += gy * gy;
        Q[3] += gx * res;
        Q[4] += gy * res;
        Q[5] += res * res;
        Q[6] += gx;
        Q[7] += gy;
        Q[8] += res;
      }
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) qs[par][wave][i][lane] = Q[i].x + Q[i].y;
    // occlusion / masks / sigma terms (every wave, same values)
    const float d1w = bilp(gd1, pw);
    const bool ok = (fw.iz > d1w - 0.1f) && (fw.u > 0.0f) && (fw.u < (float)W) && (fw.v > 0.0f) && (fw.v < (float)H);
    bool invalid = !ok || !out_lane || !fm0 || !(fm1 > 0.0f);
    float A = 1.0f, bx = 0.0f, by = 0.0f, sr0 = 0.0f;
    if (!NOSIG) {
      float hx, hy;
      sobel_cols(s0t, s0m, s0b, hx, hy);
      sr0 = bilp(gs1, pw);
      const float sg = __builtin_amdgcn_sqrtf(sr0 * sr0 + s0m * s0m);  // as pixel_terms: continuous only
      A = __builtin_amdgcn_rcpf(sg);
      const float kk = s0m * (A * A * A);
      bx = kk * hx;
      by = kk * hy;
      if (TRU) invalid = invalid || (s0m == g0min) || (s0m == g0max);
    }
    __syncthreads();  // qs[par] complete; the other buffer is free for the next unit
    if (out_lane) {
      float q[9];
#pragma unroll
      for (int i = 0; i < 9; ++i)
        q[i] = ((qs[par][0][i][lane] + qs[par][1][i][lane]) + qs[par][2][i][lane]) + qs[par][3][i][lane];
      const float A2 = A * A;
      const float Saa = A2 * q[0] + 2.0f * A * bx * q[3] + bx * bx * q[5];
      const float Sab = A2 * q[1] + A * by * q[3] + A * bx * q[4] + bx * by * q[5];
      const float Sbb = A2 * q[2] + 2.0f * A * by * q[4] + by * by * q[5];
      const float Sa = -(A * q[6] + bx * q[8]), Sb = -(A * q[7] + by * q[8]);
      const float Sar = -(A2 * q[3] + A * bx * q[5]), Sbr = -(A2 * q[4] + A * by * q[5]);
      float Jx[6], Jy[6];
      warp_jac(fw.xr, fw.yr, d, fx, fy, Jx, Jy);
      acc.add(wave, lane, Saa, Sab, Sbb, Sa, Sb, Sar, Sbr, Jx, Jy, invalid, sr0, lds_ext);
    }
  }
  acc.write_record(wave, lane, lds_ext, red, out);
}

template <int CT, bool TRU, int MODE>
__global__ __launch_bounds__(kThreads, 4) void ic_split_kernel(IterParams p) {  // 4 waves per SIMD: <= 128 VGPRs
  static_assert(MODE != 1, "combine_ICP runs on ic_reduce_kernel");
  constexpr int NQ = CT / 4, QW = NQ / 4;
  static_assert(CT % 16 == 0 && QW >= 1, "4 waves x whole channel quads");
  __shared__ float qs[2][4][9][64];
  static_assert(sizeof(qs) >= kFinScratch * sizeof(float), "finalize scratch (channel sums)");
  __shared__ float lds_ext[TRU ? 14 : 1][64];
  __shared__ float red[kRec];
  const int kb = xcd_remap(blockIdx.x, gridDim.x);
  const int b = kb / p.nbpp, jb = kb - b * p.nbpp;
  split_pass<CT, TRU, MODE>(p, b, jb, p.nbpp, qs, lds_ext, red, p.rec + (size_t)kb * kRec);

}

// ============================================================ residual-only kernel
// blockIdx.y = pose index: P poses per pair share the level's inputs; pose p
// evaluates the batch of B pairs at R[p], t[p] (its own batch-global
// truncated-sigma extrema, as one reference call per pose would).
template <bool CS1, int MODE>
__global__ __launch_bounds__(kThreads) void ic_residual_kernel(IterParams p) {
  constexpr bool ICP = MODE == 1, NOSIG = MODE == 2;
  __shared__ float red[4][16];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int bid = xcd_remap(blockIdx.x, p.nblocks);
  const int pi = blockIdx.y;
  const int tx = bid % p.tiles_x;
  const int rest = bid / p.tiles_x;
  const int ty = rest % p.tiles_y;
  const int b = rest / p.tiles_y;
  const int W = p.W, H = p.H, HW = H * W, C = p.C;
  const bool tru = (p.flags & DPFT_REMOVE_TRU_SIGMA) != 0;
  const bool c4 = (p.flags & DPFT_FEATURES_C4) != 0;
  const int fs = c4 ? 4 : 1;  // element stride of a feature channel
  const float fx = p.K[4 * b + 0], fy = p.K[4 * b + 1], cx = p.K[4 * b + 2], cy = p.K[4 * b + 3];
  float Rm[9], tv[3];
  for (int k = 0; k < 9; ++k) Rm[k] = p.R[9 * ((size_t)pi * p.B + b) + k];
  for (int k = 0; k < 3; ++k) tv[k] = p.t[3 * ((size_t)pi * p.B + b) + k];
  const float g0min = dec_ord(p.ext[0]), g0max = dec_ord(p.ext[1]);
  const float* f0b = p.f0 + (size_t)b * C * HW;
  const float* f1b = p.f1 + (size_t)b * C * HW;
  const float* s0b = p.s0 + (size_t)b * p.Cs * HW;
  const float* s1b = p.s1 + (size_t)b * p.Cs * HW;

  float sum = 0.f, ninv = 0.f;
  float mn_all = INFINITY, mn0 = INFINITY, lmn = 0.f, nmn = 0.f;
  float mx_all = -INFINITY, mx0 = -INFINITY, lmx = 0.f, nmx = 0.f;
  for (int step = 0; step < p.steps; ++step) {
    const int y = (ty * p.steps + step) * kRowsPerStep + wave, x = tx * kTileOut + lane;
    if (lane >= kTileOut || x >= W || y >= H) continue;
    const int pix = y * W + x;
    PixelFrame px;
    setup_pixel(p, b, x, y, p.invD0[(size_t)b * HW + pix], Rm, tv, fx, fy, cx, cy, px);
    float srr = 0.f, smin = INFINITY, smax = -INFINITY, sr0 = 0.f, s00 = 0.f;
    for (int c = 0; c < C; ++c) {
      if (NOSIG) {  // TrustRegionBase.forward_residuals: r = f1(warp) - f0 (algorithms.py:1919-1957)
        const float r = bil_s(chan_base(f1b, c, HW, c4), px.tp, fs) - chan_base(f0b, c, HW, c4)[(size_t)pix * fs];
        srr += r * r;
        continue;
      }
      const int cs = CS1 ? 0 : c;
      const float s0c = s0b[(size_t)cs * HW + pix];
      const float src = bil(s1b + (size_t)cs * HW, px.tp);
      if (c == 0) {
        sr0 = src;
        s00 = s0c;
      }
      smin = fminf(smin, src);
      smax = fmaxf(smax, src);
      const float r = bil_s(chan_base(f1b, c, HW, c4), px.tp, fs) - chan_base(f0b, c, HW, c4)[(size_t)pix * fs];
      const float rw = r / sqrtf(src * src + s0c * s0c);
      srr += rw * rw;
    }
    bool inv = px.invalid;
    if (tru) inv = inv || (s00 == g0min) || (s00 == g0max);
    if (ICP) {  // forward_residuals: ICP without object masks, combined occlusion (algorithms.py:765-782)
      const IcpTerm ic = icp_pixel(px.xr, px.yr, p.depth0[(size_t)b * HW + pix], Rm, tv, fx, fy, cx, cy, H, W,
                                   p.nrm1 + (size_t)b * HW, false, nullptr, p.icp_w);
      inv = inv || ic.occ;
      srr = srr + ic.r * ic.r;
    }
    sum += inv ? 0.f : srr;
    ninv += inv ? 1.f : 0.f;
    if (tru) {
      const float l = inv ? 0.f : srr, n = inv ? 0.f : 1.f;
      mn_all = fminf(mn_all, smin);
      mx_all = fmaxf(mx_all, smax);
      if (sr0 < mn0) { mn0 = sr0; lmn = l; nmn = n; } else if (sr0 == mn0) { lmn += l; nmn += n; }
      if (sr0 > mx0) { mx0 = sr0; lmx = l; nmx = n; } else if (sr0 == mx0) { lmx += l; nmx += n; }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    sum += __shfl_xor(sum, off);
    ninv += __shfl_xor(ninv, off);
    const float a0 = __shfl_xor(mn_all, off), a1 = __shfl_xor(mn0, off), a2 = __shfl_xor(lmn, off),
                a3 = __shfl_xor(nmn, off);
    mn_all = fminf(mn_all, a0);
    if (a1 < mn0) { mn0 = a1; lmn = a2; nmn = a3; } else if (a1 == mn0) { lmn += a2; nmn += a3; }
    const float b0 = __shfl_xor(mx_all, off), b1 = __shfl_xor(mx0, off), b2 = __shfl_xor(lmx, off),
                b3 = __shfl_xor(nmx, off);
    mx_all = fmaxf(mx_all, b0);
    if (b1 > mx0) { mx0 = b1; lmx = b2; nmx = b3; } else if (b1 == mx0) { lmx += b2; nmx += b3; }
  }
  if (lane == 0) {
    red[wave][L_SUM] = sum; red[wave][L_NINV] = ninv;
    red[wave][L_MN_ALL] = mn_all; red[wave][L_MN0] = mn0; red[wave][L_LMN] = lmn; red[wave][L_NMN] = nmn;
    red[wave][L_MX_ALL] = mx_all; red[wave][L_MX0] = mx0; red[wave][L_LMX] = lmx; red[wave][L_NMX] = nmx;
  }
  __syncthreads();
  if (tid == 0) {
    float* out = p.rec + ((size_t)pi * p.nblocks + bid) * kRec;
    float s = red[0][L_SUM], ni = red[0][L_NINV];
    float ma = red[0][L_MN_ALL], m0 = red[0][L_MN0], lm = red[0][L_LMN], nm = red[0][L_NMN];
    float xa = red[0][L_MX_ALL], x0v = red[0][L_MX0], lx = red[0][L_LMX], nx = red[0][L_NMX];
    for (int w = 1; w < 4; ++w) {
      s += red[w][L_SUM];
      ni += red[w][L_NINV];
      ma = fminf(ma, red[w][L_MN_ALL]);
      if (red[w][L_MN0] < m0) { m0 = red[w][L_MN0]; lm = red[w][L_LMN]; nm = red[w][L_NMN]; }
      else if (red[w][L_MN0] == m0) { lm += red[w][L_LMN]; nm += red[w][L_NMN]; }
      xa = fmaxf(xa, red[w][L_MX_ALL]);
      if (red[w][L_MX0] > x0v) { x0v = red[w][L_MX0]; lx = red[w][L_LMX]; nx = red[w][L_NMX]; }
      else if (red[w][L_MX0] == x0v) { lx += red[w][L_LMX]; nx += red[w][L_NMX]; }
    }
    st_ag(out + L_SUM, (float)(s)); st_ag(out + L_NINV, (float)(ni));
    st_ag(out + L_MN_ALL, (float)(ma)); st_ag(out + L_MN0, (float)(m0)); st_ag(out + L_LMN, (float)(lm)); st_ag(out + L_NMN, (float)(nm));
    st_ag(out + L_MX_ALL, (float)(xa)); st_ag(out + L_MX0, (float)(x0v)); st_ag(out + L_LMX, (float)(lx)); st_ag(out + L_NMX, (float)(nx));
  }
  if (block_is_last(p.ctrl + kCtlPair + pi, 1u, (uint32_t)p.nblocks)) {
    FinParams q = p.fin;
    q.rec += (size_t)pi * p.nblocks * kRec;
    q.loss_out += (size_t)pi * p.B;
    finalize_loss(q);
  }
}


// ============================================================ per-pixel debug dump
// out [B,5,H,W]: u, v, sigma_r (channel 0), sigma0 (channel 0), base-invalid
// (occlusion | masks) as 0/1.  Test / debugging only (not on the solve path).
__global__ __launch_bounds__(kThreads) void ic_debug_pixels_kernel(IterParams p, float* out) {
  const int W = p.W, H = p.H, HW = H * W;
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= p.B * HW) return;
  const int b = i / HW, pix = i - b * HW, y = pix / W, x = pix - y * W;
  const float fx = p.K[4 * b + 0], fy = p.K[4 * b + 1], cx = p.K[4 * b + 2], cy = p.K[4 * b + 3];
  float Rm[9], tv[3];
  for (int k = 0; k < 9; ++k) Rm[k] = p.R[9 * b + k];
  for (int k = 0; k < 3; ++k) tv[k] = p.t[3 * b + k];
  const float d = p.invD0[(size_t)b * HW + pix];
  const Warp w = warp_point(x, y, d, Rm, tv, fx, fy, cx, cy);
  PixelFrame px;
  setup_pixel(p, b, x, y, d, Rm, tv, fx, fy, cx, cy, px);
  float* o = out + (size_t)b * 5 * HW + pix;
  o[0] = w.u;
  o[HW] = w.v;
  o[2 * HW] = bil(p.s1 + (size_t)b * p.Cs * HW, px.tp);
  o[3 * HW] = p.s0[(size_t)b * p.Cs * HW + pix];
  o[4 * HW] = px.invalid ? 1.0f : 0.0f;
}

// The IC tracker's residual map at a pose (compute_warped_residual, algorithms.py:1919-1957):
// r_c = bilinear(f1_c, warp) - f0_c, 1e-3 on occluded / masked pixels, and the occlusion
// map -- the input of the learned M-estimator (DeepRobustEstimator, 1467-1477) and of
// its weighted loss.  One thread per pixel, every channel (NCHW or channel-quad f0 / f1).
__global__ __launch_bounds__(kThreads) void ic_residual_map_kernel(IterParams p, float* out, uint8_t* occ_out) {
  const int W = p.W, H = p.H, HW = H * W;
  const long i = (long)blockIdx.x * kThreads + threadIdx.x;
  if (i >= (long)p.B * HW) return;
  const int b = (int)(i / HW), pix = (int)(i - (long)b * HW), y = pix / W, x = pix - y * W;
  const float fx = p.K[4 * b + 0], fy = p.K[4 * b + 1], cx = p.K[4 * b + 2], cy = p.K[4 * b + 3];
  float Rm[9], tv[3];
  for (int k = 0; k < 9; ++k) Rm[k] = p.R[9 * b + k];
  for (int k = 0; k < 3; ++k) tv[k] = p.t[3 * b + k];
  const float d = p.invD0[(size_t)b * HW + pix];
  PixelFrame px;
  setup_pixel(p, b, x, y, d, Rm, tv, fx, fy, cx, cy, px);
  const bool c4 = (p.flags & DPFT_FEATURES_C4) != 0;
  const int fs = c4 ? 4 : 1;
  const float* f0b = p.f0 + (size_t)b * p.C * HW;
  const float* f1b = p.f1 + (size_t)b * p.C * HW;
  float* o = out + (size_t)b * p.C * HW + pix;
  for (int c = 0; c < p.C; ++c) {
    const float r = bil_s(chan_base(f1b, c, HW, c4), px.tp, fs) - chan_base(f0b, c, HW, c4)[(size_t)pix * fs];
    o[(size_t)c * HW] = px.invalid ? 1e-3f : r;
  }
  if (occ_out) occ_out[i] = px.invalid ? 1 : 0;
}

// NCHW -> channel-quad layout: thread i = (b, q, pixel) gathers channels 4q..4q+3
// (four coalesced plane reads) into one 16-byte store.
__global__ __launch_bounds__(kThreads) void pack_c4_kernel(const float* __restrict__ src, f32x4* __restrict__ dst,
                                                           long n, int HW) {
  const long i = (long)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const long bq = i / HW, pix = i - bq * HW;  // bq = b * C/4 + q: planes 4 bq .. 4 bq + 3
  const float* s = src + bq * 4 * HW + pix;
  dst[i] = f32x4{s[0], s[HW], s[2 * (long)HW], s[3 * (long)HW]};
}

// The same for a solve entered with NCHW features (pack_on_entry): f0 and f1 in one launch
// (blockIdx.y), four pixels per thread -- one 16-byte load from each of the quad's four
// planes, a 4 x 4 register transpose, four 16-byte stores (64 contiguous bytes per lane).
__global__ __launch_bounds__(kThreads) void pack_c4_x4_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                              f32x4* __restrict__ da, f32x4* __restrict__ db, long n,
                                                              long HW4) {
  const long i = (long)blockIdx.x * kThreads + threadIdx.x;  // (b * C/4 + q) * HW / 4 + pixel group
  if (i >= n) return;
  const f32x4* s = reinterpret_cast<const f32x4*>(blockIdx.y ? b : a);
  f32x4* o = (blockIdx.y ? db : da) + 4 * i;
  const long bq = i / HW4, g = i - bq * HW4;
  const f32x4* sp = s + bq * 4 * HW4 + g;
  const f32x4 c0 = __builtin_nontemporal_load(sp), c1 = __builtin_nontemporal_load(sp + HW4),
              c2 = __builtin_nontemporal_load(sp + 2 * HW4), c3 = __builtin_nontemporal_load(sp + 3 * HW4);
  o[0] = f32x4{c0.x, c1.x, c2.x, c3.x};
  o[1] = f32x4{c0.y, c1.y, c2.y, c3.y};
  o[2] = f32x4{c0.z, c1.z, c2.z, c3.z};
  o[3] = f32x4{c0.w, c1.w, c2.w, c3.w};
}
// (any H W or alignment: one pixel per thread, as pack_c4_kernel, f0 / f1 by blockIdx.y)
__global__ __launch_bounds__(kThreads) void pack_c4_pair_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                                f32x4* __restrict__ da, f32x4* __restrict__ db, long n,
                                                                long HW) {
  const long i = (long)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const long bq = i / HW, pix = i - bq * HW;
  const float* s = (blockIdx.y ? b : a) + bq * 4 * HW + pix;
  (blockIdx.y ? db : da)[i] = f32x4{s[0], s[HW], s[2 * HW], s[3 * HW]};
}

// NHWC (channels_last) -> channel-quad layout: thread r of pair row b = blockIdx.y reads
// the 16-byte quad r of the pair's [HW][C] block (a linear, coalesced read) and writes it
// to plane q = r % Q at pixel r / Q (64 lanes = 64 / Q pixels x Q planes: one 128-byte run
// per plane for Q = 8).
__global__ __launch_bounds__(kThreads) void pack_c4_nhwc_kernel(const f32x4* __restrict__ src,
                                                                f32x4* __restrict__ dst, uint32_t n, uint32_t Q,
                                                                uint32_t HW) {
  const uint32_t r = blockIdx.x * kThreads + threadIdx.x;
  if (r >= n) return;
  const size_t base = (size_t)blockIdx.y * n;
  const uint32_t pix = r / Q, q = r - pix * Q;
  dst[base + (size_t)q * HW + pix] = __builtin_nontemporal_load(src + base + r);
}

// sigma0 batch-global min / max (algorithms.py:1976-1977).  Per-workgroup
// partials, the last workgroup reduces them in a fixed order (no atomics on data).
__device__ void minmax_body(const float* __restrict__ s, size_t n, uint32_t* ctrl, int slot, float* part,
                            uint32_t* done) {
  __shared__ float sm[2][4];
  float mn = INFINITY, mx = -INFINITY;
  // 16-byte loads, four in flight per thread per round (a scalar grid-stride loop
  // waits one memory latency per element: 17.6 us for 9.8 MB at level 0)
  const size_t head = std::min<size_t>(((16 - (reinterpret_cast<uintptr_t>(s) & 15)) & 15) / 4, n);
  const size_t n4 = (n - head) / 4;
  const f32x4* s4 = reinterpret_cast<const f32x4*>(s + head);
  const size_t stride = (size_t)gridDim.x * kThreads;
  const size_t t0 = (size_t)blockIdx.x * kThreads + threadIdx.x;
  size_t i = t0;
  for (; i + (kMMLoads - 1) * stride < n4; i += kMMLoads * stride) {
    f32x4 v[kMMLoads];
#pragma unroll
    for (int u = 0; u < kMMLoads; ++u) v[u] = __builtin_nontemporal_load(s4 + i + u * stride);
#pragma unroll
    for (int u = 0; u < kMMLoads; ++u) {
      mn = fminf(mn, fminf(fminf(v[u].x, v[u].y), fminf(v[u].z, v[u].w)));
      mx = fmaxf(mx, fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w)));
    }
  }
  for (; i < n4; i += stride) {
    const f32x4 v = s4[i];
    mn = fminf(mn, fminf(fminf(v.x, v.y), fminf(v.z, v.w)));
    mx = fmaxf(mx, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
  }
  if (t0 < head) {  // unaligned head
    mn = fminf(mn, s[t0]);
    mx = fmaxf(mx, s[t0]);
  }
  for (size_t j = head + n4 * 4 + t0; j < n; j += stride) {  // tail
    mn = fminf(mn, s[j]);
    mx = fmaxf(mx, s[j]);
  }
  for (int off = 32; off > 0; off >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, off));
    mx = fmaxf(mx, __shfl_xor(mx, off));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    sm[0][wave] = mn;
    sm[1][wave] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    st_ag(part + 2 * blockIdx.x, fminf(fminf(sm[0][0], sm[0][1]), fminf(sm[0][2], sm[0][3])));
    st_ag(part + 2 * blockIdx.x + 1, fmaxf(fmaxf(sm[1][0], sm[1][1]), fmaxf(sm[1][2], sm[1][3])));
  }
  if (!block_is_last(done, 1u, gridDim.x)) return;
  if (threadIdx.x < 64) {
    mn = INFINITY;
    mx = -INFINITY;
    for (int k = threadIdx.x; k < (int)gridDim.x; k += 64) {
      mn = fminf(mn, ld_ag(part + 2 * k));
      mx = fmaxf(mx, ld_ag(part + 2 * k + 1));
    }
    for (int off = 32; off > 0; off >>= 1) {
      mn = fminf(mn, __shfl_xor(mn, off));
      mx = fmaxf(mx, __shfl_xor(mx, off));
    }
    if (threadIdx.x == 0) {
      ctrl[slot] = enc_ord(mn);
      ctrl[slot + 1] = enc_ord(mx);
    }
  }
}

__global__ __launch_bounds__(kThreads) void minmax_kernel(const float* __restrict__ s, size_t n, uint32_t* ctrl,
                                                          int slot) {
  minmax_body(s, n, ctrl, slot, reinterpret_cast<float*>(ctrl + kCtlPart), ctrl + kCtlMMDone);
}

// Every level's sigma0 extrema in one launch (blockIdx.y = level): one pose-independent
// pre-pass per pyramid solve instead of one launch per level.
// DPFT_GROUP: blockIdx.y = level * groups + batch, each batch's extrema over its own
// pairs into its own slot word pair (one call = one batch: exactly the per-level pass).
struct MMLevels {
  const float* s[4];
  size_t n[4];  // floats per batch
  int slot[4];
  int groups;
};
__global__ __launch_bounds__(kThreads) void minmax_levels_kernel(MMLevels a, uint32_t* ctrl) {
  const int l = blockIdx.y / a.groups, g = blockIdx.y - l * a.groups;
  minmax_body(a.s[l] + (size_t)g * a.n[l], a.n[l], ctrl, a.slot[l] + 2 * g,
              reinterpret_cast<float*>(ctrl + kCtlPart) + 2 * blockIdx.y * gridDim.x,
              ctrl + (a.groups > 1 ? kCtlGMMDone : kCtlMMDoneL) + blockIdx.y);
}

// ============================================================ depth preprocessing
// LeastSquareTracking._preprocess (LeastSquareTracking.py:653-661, 669-670):
// invD = clamp(1 / depth, 0, 10); zero the batch-global min, then the max;
// ImagePyramids(pool='max') (algorithms.py:1201-1219) of invD (and of the raw
// depth for ICP).  Bit-exact: IEEE division, NaN-propagating clamp and max.
__device__ __forceinline__ float invd_of(float d) {
  const float x = 1.0f / d;
  return x < 0.0f ? 0.0f : (x > 10.0f ? 10.0f : x);  // torch.clamp (NaN stays NaN)
}

__global__ __launch_bounds__(kThreads) void invd_minmax_kernel(const float* __restrict__ depth, size_t n,
                                                               uint32_t* ctrl) {
  __shared__ float sm[2][4];
  float mn = INFINITY, mx = -INFINITY;
  const size_t stride = (size_t)gridDim.x * kThreads;
  for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    const float v = invd_of(depth[i]);
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  for (int off = 32; off > 0; off >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, off));
    mx = fmaxf(mx, __shfl_xor(mx, off));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    sm[0][wave] = mn;
    sm[1][wave] = mx;
  }
  __syncthreads();
  float* part = reinterpret_cast<float*>(ctrl + kCtlPart);
  if (threadIdx.x == 0) {
    st_ag(part + 2 * blockIdx.x, fminf(fminf(sm[0][0], sm[0][1]), fminf(sm[0][2], sm[0][3])));
    st_ag(part + 2 * blockIdx.x + 1, fmaxf(fmaxf(sm[1][0], sm[1][1]), fmaxf(sm[1][2], sm[1][3])));
  }
  if (!block_is_last(ctrl + kCtlMMDone, 1u, gridDim.x)) return;
  if (threadIdx.x < 64) {
    mn = INFINITY;
    mx = -INFINITY;
    for (int k = threadIdx.x; k < (int)gridDim.x; k += 64) {
      mn = fminf(mn, ld_ag(part + 2 * k));
      mx = fmaxf(mx, ld_ag(part + 2 * k + 1));
    }
    for (int off = 32; off > 0; off >>= 1) {
      mn = fminf(mn, __shfl_xor(mn, off));
      mx = fmaxf(mx, __shfl_xor(mx, off));
    }
    if (threadIdx.x == 0) {
      // the max is taken after the min pixels were zeroed (LeastSquareTracking.py:658-661)
      const float mx2 = (mx == mn) ? 0.0f : mx;
      ctrl[kCtlMin] = enc_ord(mn);
      ctrl[kCtlMax] = enc_ord(mx2);
    }
  }
}

struct PyrOut {
  float* invd[4];
  float* depth[4];
};

// blockIdx.y = level l: each thread writes one level-l pixel, the max over its
// 2^l x 2^l block (MaxPool2d(2^l, 2^l): floor-sized output, remainder ignored).
__global__ __launch_bounds__(kThreads) void invd_pyramid_kernel(const float* __restrict__ depth, int B, int H, int W,
                                                                const uint32_t* __restrict__ ctrl, PyrOut out) {
  const int l = blockIdx.y, k = 1 << l;
  const int Hl = H / k, Wl = W / k;
  const long i = (long)blockIdx.x * kThreads + threadIdx.x;
  if (i >= (long)B * Hl * Wl) return;
  const int b = (int)(i / ((long)Hl * Wl)), rem = (int)(i - (long)b * Hl * Wl), y = rem / Wl, x = rem - y * Wl;
  const float gmin = dec_ord(ctrl[kCtlMin]), gmax = dec_ord(ctrl[kCtlMax]);
  const float* db = depth + (size_t)b * H * W;
  float mi = -INFINITY, md = -INFINITY;
  bool nan_i = false, nan_d = false;
  for (int yy = y * k; yy < y * k + k; ++yy)
    for (int xx = x * k; xx < x * k + k; ++xx) {
      const float d = db[yy * W + xx];
      float v = invd_of(d);
      if (v == gmin || v == gmax) v = 0.0f;
      nan_i |= v != v;
      nan_d |= d != d;
      mi = fmaxf(mi, v);
      md = fmaxf(md, d);
    }
  const size_t o = (size_t)b * Hl * Wl + rem;
  out.invd[l][o] = nan_i ? NAN : mi;
  if (out.depth[l]) out.depth[l][o] = nan_d ? NAN : md;
}

// ------------------------------------------------------------------ host side
struct Geometry {
  int tiles_x, tiles_y, steps, nblocks, per_pair;
};

Geometry plan(const DpftLevelDesc& d) {
  Geometry g;
  g.tiles_x = (d.W + kTileW - 3) / (kTileW - 2);  // 62 output columns per tile (2 halo lanes)
  const int row_groups = (d.H + kRowsPerStep - 1) / kRowsPerStep;
  int steps = kMaxSteps;
  // prefer >= 2048 workgroups (8 per CU) before taller tiles
  while (steps > 1 && (long)g.tiles_x * ((row_groups + steps - 1) / steps) * d.B < 2048) steps >>= 1;
  g.steps = steps;
  g.tiles_y = (row_groups + steps - 1) / steps;
  g.per_pair = g.tiles_x * g.tiles_y;
  g.nblocks = g.per_pair * d.B;
  return g;
}

int check_desc(const DpftLevelDesc* d) {
  if (!d) return fail(DPFT_E_INVALID, "null descriptor");
  if (d->B < 1 || d->C < 1 || d->H < 2 || d->W < 2)
    return fail(DPFT_E_INVALID, "bad shape B=%d C=%d H=%d W=%d", d->B, d->C, d->H, d->W);
  if (d->Cs != 1 && d->Cs != d->C) return fail(DPFT_E_INVALID, "Cs must be 1 or C (got %d, C=%d)", d->Cs, d->C);
  if ((long)d->H * d->W >= (1L << 30)) return fail(DPFT_E_INVALID, "level too large");
  if (d->B > kMaxPairs) return fail(DPFT_E_INVALID, "B=%d exceeds %d pairs per call", d->B, kMaxPairs);
  if ((d->flags & DPFT_COMBINE_ICP) && !(d->icp_weight == d->icp_weight))
    return fail(DPFT_E_INVALID, "icp_weight is NaN");
  if (((d->flags & DPFT_EXT_SLOT_MASK) >> DPFT_EXT_SLOT_SHIFT) > (uint32_t)kMaxExtSlots)
    return fail(DPFT_E_INVALID, "extrema slot out of range");
  if ((d->flags & DPFT_EXTREMA_READY) && !(d->flags & DPFT_EXT_SLOT_MASK))
    return fail(DPFT_E_INVALID, "EXTREMA_READY needs an extrema slot (DPFT_EXT_SLOT)");
  if ((d->flags & DPFT_NO_UNCERTAINTY) && (d->flags & (DPFT_REMOVE_TRU_SIGMA | DPFT_COMBINE_ICP)))
    return fail(DPFT_E_INVALID, "NO_UNCERTAINTY (IC tracker) excludes REMOVE_TRU_SIGMA and COMBINE_ICP");
  if ((d->flags & DPFT_FEATURES_C4) && (d->C % 4 != 0 || (d->Cs != 1 && !(d->flags & DPFT_NO_UNCERTAINTY))))
    return fail(DPFT_E_INVALID, "FEATURES_C4 needs C %% 4 == 0 and one sigma plane (C=%d, Cs=%d)", d->C, d->Cs);
  const int gs = (int)((d->flags & DPFT_GROUP_MASK) >> DPFT_GROUP_SHIFT);
  if (gs != 0 && gs < d->B) {
    if (d->B % gs != 0 || d->B / gs > kMaxGroups)
      return fail(DPFT_E_INVALID, "DPFT_GROUP(%d): B=%d must be a multiple of it, at most %d batches", gs, d->B,
                  kMaxGroups);
  }
  return DPFT_OK;
}

// pairs per independent batch of the call (DPFT_GROUP; B = one batch)
int group_of(const DpftLevelDesc& d) {
  const int gs = (int)((d.flags & DPFT_GROUP_MASK) >> DPFT_GROUP_SHIFT);
  return (gs == 0 || gs >= d.B) ? d.B : gs;
}
// ctrl word of batch 0's sigma0 extrema for this call (batch g: + 2 g)
int ext_word(const DpftLevelDesc& d) {
  const int xslot = (int)((d.flags & DPFT_EXT_SLOT_MASK) >> DPFT_EXT_SLOT_SHIFT);  // 0: none
  if (group_of(d) == d.B) return xslot ? kCtlExtSlots + 2 * (xslot - 1) : kCtlMin;
  return kCtlGExt + 2 * kMaxGroups * (xslot ? xslot - 1 : kMaxExtSlots);
}

int check_tensors(const DpftLevelTensors* t, uint32_t flags = 0) {
  if (!t || !t->f0 || !t->f1 || !t->invD0 || !t->invD1 || !t->K)
    return fail(DPFT_E_INVALID, "null tensor pointer");
  if (!(flags & DPFT_NO_UNCERTAINTY) && (!t->s0 || !t->s1)) return fail(DPFT_E_INVALID, "null sigma pointer");
  if ((flags & DPFT_COMBINE_ICP) && (!t->depth0 || !t->depth1))
    return fail(DPFT_E_INVALID, "COMBINE_ICP needs depth0 and depth1");
  if (t->weights && !(flags & DPFT_NO_UNCERTAINTY))
    return fail(DPFT_E_INVALID, "per-pixel weights are the IC tracker's M-estimator (NO_UNCERTAINTY only)");
  return DPFT_OK;
}

// workspace: [ctrl][pair records B x kPRec fp64][workgroup records nblocks x kRec fp32]
size_t prec_bytes(const DpftLevelDesc& d) { return ((size_t)d.B * kPRec * sizeof(double) + 255) & ~(size_t)255; }

// reduce-kernel record slots: B * nbpp <= max(kMaxGrid, B)
size_t rec_bytes(const DpftLevelDesc& d) {
  const Geometry g = plan(d);
  const size_t slots = std::max<size_t>(std::max<size_t>(kMaxGrid, d.B), (size_t)g.nblocks);
  return (slots * kRec * sizeof(float) + 255) & ~(size_t)255;
}

// COMBINE_ICP: frame-1 normal + depth map [B,H,W,4] and the ICP records between the pair
// records and the workgroup records (the latter grow with the number of poses of a residual
// call)
size_t nrm_bytes(const DpftLevelDesc& d) {
  if (!(d.flags & DPFT_COMBINE_ICP)) return 0;
  // the map, then the ICP records (icp_records_kernel: one per reduce workgroup slot)
  const size_t slots = std::max<size_t>(kMaxGrid, d.B);
  return (((size_t)d.B * 4 * d.H * d.W * sizeof(float) + 255) & ~(size_t)255) + slots * kIcpSub * kIcpRec * sizeof(float);
}
size_t icp_rec_offset(const DpftLevelDesc& d) {
  return kCtrlBytes + prec_bytes(d) + (((size_t)d.B * 4 * d.H * d.W * sizeof(float) + 255) & ~(size_t)255);
}

// every entry point's own regions: control words, pair / ICP / workgroup records
size_t ws_core(const DpftLevelDesc& d) {
  return kCtrlBytes + prec_bytes(d) + ((nrm_bytes(d) + 255) & ~(size_t)255) + rec_bytes(d);
}
// NCHW features handed to a solve (the reference's layout, algorithms.py:611-723) are packed
// once on entry into the workspace's channel-quad copy, and the level's iterations run the
// channel-quad kernels on it: where those are the marching / split kernels (C % 16 == 0) and
// the level has one sigma plane (or none), from two iterations on.  The NCHW kernel (the tile
// path) reads f1's taps channel plane by channel plane at half the rate.
bool packs_on_entry(const DpftLevelDesc& d) {
  return !(d.flags & DPFT_FEATURES_C4) && d.C % 16 == 0 && (d.Cs == 1 || (d.flags & DPFT_NO_UNCERTAINTY)) &&
         d.iters >= 2;
}
size_t pack_plane_bytes(const DpftLevelDesc& d) {
  return ((size_t)d.B * d.C * d.H * d.W * sizeof(float) + 255) & ~(size_t)255;
}
// + the packed f0 / f1 of a solve entered with NCHW features (packs_on_entry)
size_t ws_need(const DpftLevelDesc& d) { return ws_core(d) + (packs_on_entry(d) ? 2 * pack_plane_bytes(d) : 0); }
size_t nrm_offset(const DpftLevelDesc& d) { return kCtrlBytes + prec_bytes(d); }
size_t rec_offset(const DpftLevelDesc& d) { return kCtrlBytes + prec_bytes(d) + ((nrm_bytes(d) + 255) & ~(size_t)255); }

// residual evaluation of P poses: P x nblocks records (normal map after them)
size_t ws_need_poses(const DpftLevelDesc& d, int P) {
  const Geometry g = plan(d);
  const size_t rec = ((size_t)P * g.nblocks * kRec * sizeof(float) + 255) & ~(size_t)255;
  return rec_offset(d) + std::max(rec, rec_bytes(d));
}

// Image sizes whose tap divisor (n - 1) / 2 tools/div_check.c verifies div_const on for all
// 2^32 floats (mode 0): every level of 640x480 and of 160x120.  Other sizes take the IEEE
// division (make_taps_xy<false>).
constexpr int kVerifiedTapSizes[] = {640, 320, 160, 80, 40, 20, 480, 240, 120, 60, 30, 15};
bool tap_div_verified(int n) {
  for (int v : kVerifiedTapSizes)
    if (n == v) return true;
  return false;
}

IterParams make_params(const DpftLevelDesc& d, const DpftLevelTensors& tt, const Geometry& g, const float* R,
                       const float* t, void* ws) {
  IterParams p;
  p.f0 = tt.f0;
  p.f1 = tt.f1;
  p.s0 = tt.s0;
  p.s1 = tt.s1;
  p.invD0 = tt.invD0;
  p.invD1 = tt.invD1;
  p.mask0 = tt.mask0;
  p.mask1 = tt.mask1;
  p.wgt = tt.weights;
  p.depth0 = tt.depth0;
  p.depth1 = tt.depth1;
  p.nrm1 = (d.flags & DPFT_COMBINE_ICP) ? reinterpret_cast<const f32x4*>(static_cast<char*>(ws) + nrm_offset(d))
                                        : nullptr;
  p.icp_rec = (d.flags & DPFT_COMBINE_ICP) ? reinterpret_cast<float*>(static_cast<char*>(ws) + icp_rec_offset(d))
                                           : nullptr;
  p.icp_w = d.icp_weight;
  p.K = tt.K;
  p.R = R;
  p.t = t;
  p.B = d.B;
  p.C = d.C;
  p.Cs = d.Cs;
  p.H = d.H;
  p.W = d.W;
  p.tiles_x = g.tiles_x;
  p.tiles_y = g.tiles_y;
  p.steps = g.steps;
  p.nblocks = g.nblocks;
  p.flags = d.flags;
  p.ctrl = reinterpret_cast<uint32_t*>(ws);
  p.ext = p.ctrl + ext_word(d);
  p.rec = reinterpret_cast<float*>(static_cast<char*>(ws) + rec_offset(d));
  // rows per step of the reduce kernel (4 waves x rows per lane of the instantiation launched)
  p.rps = 4 * ((d.flags & DPFT_FEATURES_C4) ? kRPL4 : (d.Cs == 1 || (d.flags & DPFT_NO_UNCERTAINTY)) ? kRPL : 1);
  p.row_groups = (d.H + p.rps - 1) / p.rps;
  p.per_pair = g.tiles_x * p.row_groups;
  p.nbpp = 0;  // set at launch from the kernel's resident capacity
  p.round_wg = 0;
  p.fin_on = 0;
  p.reverse = 0;
  p.skew = kMarchSkew;
  p.rc_taps = tap_div_verified(d.W) && tap_div_verified(d.H);
  memset(&p.fin, 0, sizeof(p.fin));
  p.fin.rec = p.rec;
  p.fin.prec = reinterpret_cast<double*>(static_cast<char*>(ws) + kCtrlBytes);
  p.fin.pair_cnt = p.ctrl + kCtlPair;
  p.fin.group = group_of(d);
  p.fin.done_cnt = p.ctrl + (p.fin.group < d.B ? kCtlGDone : kCtlDone);
  p.fin.nblocks = g.nblocks;
  p.fin.per_pair = g.per_pair;
  p.fin.HW = d.H * d.W;
  p.fin.flags = d.flags;
  p.fin.status = tt.status;
  p.fin.B = d.B;
  return p;
}

int hip_check(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(DPFT_E_HIP, "%s: %s", what, hipGetErrorString(e));
  return DPFT_OK;
}

int minmax_into(const float* src, size_t n, uint32_t* ctrl, int slot, hipStream_t st) {
  const int grid = (int)std::min<size_t>((n + kThreads * 16 - 1) / (kThreads * 16), kMMGrid);
  hipLaunchKernelGGL(minmax_kernel, dim3(grid), dim3(kThreads), 0, st, src, n, ctrl, slot);
  return hip_check("minmax_kernel");
}

// Extrema of `groups` consecutive batches of n floats each in one launch (minmax_levels_kernel
// with one level, blockIdx.y = batch): batch g's (min, max) into ctrl[word + 2 g], ctrl[word + 2 g + 1].
int minmax_batches(const float* src, size_t n, int groups, uint32_t* ctrl, int word, hipStream_t st) {
  MMLevels a;
  for (int l = 0; l < 4; ++l) {
    a.s[l] = src;
    a.n[l] = n;
    a.slot[l] = word;
  }
  a.groups = groups;
  const int grid = (int)std::max<size_t>(
      1, std::min<size_t>(std::min<size_t>((n + kThreads * 16 - 1) / (kThreads * 16), kMMGrid),
                          (size_t)kMaxMMBlocks / (size_t)groups));
  hipLaunchKernelGGL(minmax_levels_kernel, dim3(grid, groups), dim3(kThreads), 0, st, a, ctrl);
  return hip_check("minmax_levels_kernel (batches)");
}

// Pose-independent per-level pre-passes (first iteration of a level):
// sigma0 batch extrema (truncated sigma), depth1 batch extrema + normal map (ICP).
int launch_minmax(const DpftLevelDesc& d, const DpftLevelTensors& tt, void* ws, hipStream_t st) {
  uint32_t* ctrl = reinterpret_cast<uint32_t*>(ws);
  int rc;
  if ((d.flags & DPFT_REMOVE_TRU_SIGMA) && !(d.flags & DPFT_EXTREMA_READY)) {
    const int gs = group_of(d);  // one extremum pair per independent batch (DPFT_GROUP)
    const size_t n = (size_t)gs * d.Cs * d.H * d.W;
    if (gs < d.B) {
      if ((rc = minmax_batches(tt.s0, n, d.B / gs, ctrl, ext_word(d), st))) return rc;
    } else if ((rc = minmax_into(tt.s0, n, ctrl, ext_word(d), st))) {
      return rc;
    }
  }
  if (d.flags & DPFT_COMBINE_ICP) {
    // depth1 min / max per independent batch (algorithms.py:2168 compares against the
    // whole batch the call holds), then frame 1's normal map
    const int gs = group_of(d);
    const int word = gs < d.B ? kCtlGD1 : kCtlD1Min;
    if (gs < d.B) {  // every batch in one launch (blockIdx.y = batch)
      if ((rc = minmax_batches(tt.depth1, (size_t)gs * d.H * d.W, d.B / gs, ctrl, word, st))) return rc;
    } else if ((rc = minmax_into(tt.depth1, (size_t)d.B * d.H * d.W, ctrl, word, st))) {
      return rc;
    }
    const int rpr = nrm_rows(d.B, d.H, d.W);
    const size_t waves = (size_t)d.B * ((d.H + rpr - 1) / rpr) * ((d.W + kTileOut - 1) / kTileOut);
    f32x4* nrm = reinterpret_cast<f32x4*>(static_cast<char*>(ws) + nrm_offset(d));
    hipLaunchKernelGGL(icp_normals_kernel, dim3((unsigned)((waves + kThreads / 64 - 1) / (kThreads / 64))),
                       dim3(kThreads), 0, st, tt.depth1, tt.K, d.B, d.H, d.W, ctrl + word, gs, nrm);
    if ((rc = hip_check("icp_normals_kernel"))) return rc;
  }
  return DPFT_OK;
}

// Workgroups of `kernel` the current device holds at once (cached per kernel and device).
int resident_blocks(const void* kernel, int threads = kThreads) {
  struct Entry {
    const void* k;
    int dev, n;
  };
  static std::mutex mu;
  static std::vector<Entry> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lock(mu);
  for (const Entry& e : cache)
    if (e.k == kernel && e.dev == dev) return e.n;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  const int n = std::max(1, std::min(per_cu * cus, kMaxGrid));
  cache.push_back({kernel, dev, n});
  return n;
}

// combine_ICP through its own pass: the records of icp_records_kernel for the reduce launch's
// B x nbpp workgroup slots, added by the launch's pair reduction (p.fin.icp_rec)
int launch_icp_records(IterParams& p, hipStream_t st) {
  // S workgroups per slot, each with at least 8 pixels per thread
  p.fin.icp_sub = std::max(1, std::min(kIcpSub, (int)((long)p.H * p.W / ((long)p.nbpp * kThreads * 8))));
  hipLaunchKernelGGL(icp_records_kernel, dim3(p.B * p.nbpp * p.fin.icp_sub), dim3(kThreads), 0, st, p, p.icp_rec);
  p.fin.icp_rec = p.icp_rec;
  return hip_check("icp_records_kernel");
}

template <int CT, bool CS1, bool TRU, int MODE, bool C4 = false>
int launch_reduce_k(IterParams p, hipStream_t st, bool icp_pass = false) {
  const void* k = reinterpret_cast<const void*>(&ic_reduce_kernel<CT, CS1, TRU, MODE, C4>);
  const int cap = resident_blocks(k);
  if (cap <= 0) return fail(DPFT_E_HIP, "occupancy query failed");
  p.nbpp = std::max(1, std::min(cap / p.B, p.per_pair));  // one dispatch round
  if ((long)p.B * p.nbpp > kMaxGrid) p.nbpp = std::max(1, kMaxGrid / p.B);
  if (C4 && CT > 0 && kMarchMinRows > 0) {  // marching: at most one wave per kMarchMinRows units
    constexpr int mr = kMarchMinRows > 0 ? kMarchMinRows : 1;
    const long waves = ((long)p.tiles_x * p.H + mr - 1) / mr;
    p.nbpp = std::max(1, std::min(p.nbpp, (int)((waves + 3) / 4)));
  }
  p.round_wg = cap / 8;
  p.fin.nbpp = p.nbpp;
  int rc;
  if (icp_pass && (rc = launch_icp_records(p, st))) return rc;
  // the finalize runs in-kernel (last-workgroup handshake, fin_on)
  hipLaunchKernelGGL((ic_reduce_kernel<CT, CS1, TRU, MODE, C4>), dim3(p.B * p.nbpp), dim3(kThreads), 0, st, p);
  return DPFT_OK;
}

template <int CT, bool CS1>
int launch_reduce_t(const IterParams& p, hipStream_t st) {
  const bool tru = (p.flags & DPFT_REMOVE_TRU_SIGMA) != 0;
  if (p.flags & DPFT_NO_UNCERTAINTY) {
    if constexpr (CS1) return launch_reduce_k<CT, true, false, 2>(p, st);
    else return fail(DPFT_E_INVALID, "internal: no IC instantiation for Cs=C");
  }
  if (p.flags & DPFT_COMBINE_ICP) {
    if constexpr (CS1 || CT == 0)
      return tru ? launch_reduce_k<CT, CS1, true, 1>(p, st) : launch_reduce_k<CT, CS1, false, 1>(p, st);
    else
      return fail(DPFT_E_INVALID, "internal: no ICP instantiation for C=%d, Cs=C", CT);
  }
  return tru ? launch_reduce_k<CT, CS1, true, 0>(p, st) : launch_reduce_k<CT, CS1, false, 0>(p, st);
}

template <int CT, bool TRU, int MODE>
int launch_split(IterParams p, hipStream_t st, bool icp_pass = false) {
  const void* k = reinterpret_cast<const void*>(&ic_split_kernel<CT, TRU, MODE>);
  const int cap = resident_blocks(k);
  if (cap <= 0) return fail(DPFT_E_HIP, "occupancy query failed");
  const int units = p.tiles_x * p.H;
  p.nbpp = std::max(1, std::min(cap / p.B, units));
  p.fin.nbpp = p.nbpp;
  int rc;
  if (icp_pass && (rc = launch_icp_records(p, st))) return rc;
  // Many small workgroups finish together here: the last-block handshake would
  // serialise B * nbpp atomics on B counters, so the finalize is its own launch
  // (B workgroups, the kernel boundary orders the records).
  const bool fin = p.fin_on != 0;
  p.fin_on = 0;
  hipLaunchKernelGGL((ic_split_kernel<CT, TRU, MODE>), dim3(p.B * p.nbpp), dim3(kThreads), 0, st, p);
  if (fin) hipLaunchKernelGGL(finalize_kernel, dim3(p.B), dim3(kThreads), 0, st, p.fin);
  return DPFT_OK;
}

template <int CT>
int launch_reduce_c4(const IterParams& p, hipStream_t st) {
  const bool tru = (p.flags & DPFT_REMOVE_TRU_SIGMA) != 0;
  if constexpr (CT > 0 && CT % 16 == 0) {
    uint32_t sched = p.flags & DPFT_SCHED_MASK;
    if (sched == DPFT_SCHED_AUTO)  // coarse levels (few pixels per pair): the channel-split kernel
      sched = ((long)p.H * p.W <= kSplitMaxPixels && (long)p.B * p.H * p.W <= kSplitMaxLaunchPixels)
                  ? DPFT_SCHED_SPLIT : DPFT_SCHED_MARCH;
    // combine_ICP: the U_IC kernels plus the point-to-plane term's own pass (icp_records_kernel)
    const bool icp = (p.flags & DPFT_COMBINE_ICP) != 0;
    if (!p.wgt) {  // M-estimator weights: ic_reduce_kernel
      if (sched == DPFT_SCHED_SPLIT) {
        if (p.flags & DPFT_NO_UNCERTAINTY) return launch_split<CT, false, 2>(p, st);
        return tru ? launch_split<CT, true, 0>(p, st, icp) : launch_split<CT, false, 0>(p, st, icp);
      }
    }
    if (icp)
      return tru ? launch_reduce_k<CT, true, true, 0, true>(p, st, true)
                 : launch_reduce_k<CT, true, false, 0, true>(p, st, true);
  }
  if (p.flags & DPFT_NO_UNCERTAINTY) return launch_reduce_k<CT, true, false, 2, true>(p, st);
  if constexpr (!(CT > 0 && CT % 16 == 0)) {  // (C % 16 == 0: the ICP pass above, no fused instance)
    if (p.flags & DPFT_COMBINE_ICP)
      return tru ? launch_reduce_k<CT, true, true, 1, true>(p, st) : launch_reduce_k<CT, true, false, 1, true>(p, st);
  }
  return tru ? launch_reduce_k<CT, true, true, 0, true>(p, st) : launch_reduce_k<CT, true, false, 0, true>(p, st);
}

int launch_reduce(const IterParams& p, hipStream_t st) {
  int rc;
  if (p.flags & DPFT_FEATURES_C4) {
    rc = p.C == 32 ? launch_reduce_c4<32>(p, st) : p.C == 16 ? launch_reduce_c4<16>(p, st) : launch_reduce_c4<0>(p, st);
  } else if (p.Cs == 1 || (p.flags & DPFT_NO_UNCERTAINTY)) {
    switch (p.C) {
      case 8: rc = launch_reduce_t<8, true>(p, st); break;
      case 16: rc = launch_reduce_t<16, true>(p, st); break;
      case 32: rc = launch_reduce_t<32, true>(p, st); break;
      default: rc = launch_reduce_t<0, true>(p, st); break;
    }
  } else {
    if (p.flags & DPFT_COMBINE_ICP) {
      rc = launch_reduce_t<0, false>(p, st);
    } else {
      switch (p.C) {
        case 8: rc = launch_reduce_t<8, false>(p, st); break;
        case 32: rc = launch_reduce_t<32, false>(p, st); break;
        default: rc = launch_reduce_t<0, false>(p, st); break;
      }
    }
  }
  if (rc) return rc;
  return hip_check("ic_reduce_kernel");
}

int iterate_impl(const DpftLevelDesc* desc, const DpftLevelTensors* tt, float* R, float* t, float* jtj_out,
                 float* jtr_out, int32_t* invalid_out, int first, void* ws, size_t ws_bytes, hipStream_t st) {
  int rc = check_desc(desc);
  if (rc) return rc;
  if ((rc = check_tensors(tt, desc->flags))) return rc;
  if (!R || !t || !ws) return fail(DPFT_E_INVALID, "null pose / workspace");
  if (ws_bytes < ws_core(*desc)) return fail(DPFT_E_WORKSPACE, "workspace %zu < %zu", ws_bytes, ws_core(*desc));
  const Geometry g = plan(*desc);
  if ((first & DPFT_ITER_FIRST) && (rc = launch_minmax(*desc, *tt, ws, st))) return rc;
  IterParams p = make_params(*desc, *tt, g, R, t, ws);
  p.reverse = (first & DPFT_ITER_REVERSE) ? 1 : 0;
  p.fin_on = 1;
  p.fin.no_update = (first & DPFT_ITER_NO_UPDATE) ? 1 : 0;
  p.fin.R = R;
  p.fin.t = t;
  p.fin.jtj_out = jtj_out;
  p.fin.jtr_out = jtr_out;
  p.fin.invalid_out = invalid_out;
  return launch_reduce(p, st);
}

// f0 and f1 [B,C,H,W] -> channel-quad copies in the workspace (packs_on_entry), one launch
int pack_on_entry(const DpftLevelDesc& d, DpftLevelDesc& dc, DpftLevelTensors& tc, void* ws, size_t ws_bytes,
                  hipStream_t st) {
  if (ws_bytes < ws_need(d)) return fail(DPFT_E_WORKSPACE, "workspace %zu < %zu", ws_bytes, ws_need(d));
  if (!tc.f0 || !tc.f1) return fail(DPFT_E_INVALID, "null tensor pointer");
  f32x4* p0 = reinterpret_cast<f32x4*>(static_cast<char*>(ws) + ws_core(d));
  f32x4* p1 = reinterpret_cast<f32x4*>(static_cast<char*>(ws) + ws_core(d) + pack_plane_bytes(d));
  const long HW = (long)d.H * d.W, quads = (long)d.B * (d.C / 4);
  const bool x4 = HW % 4 == 0 && ((uintptr_t)tc.f0 % 16) == 0 && ((uintptr_t)tc.f1 % 16) == 0;
  const long n = x4 ? quads * (HW / 4) : quads * HW;
  if ((n + kThreads - 1) / kThreads > 0x7fffffffL) return fail(DPFT_E_INVALID, "level too large to pack on entry");
  const dim3 grid((unsigned)((n + kThreads - 1) / kThreads), 2);
  if (x4)
    hipLaunchKernelGGL(pack_c4_x4_kernel, grid, dim3(kThreads), 0, st, tc.f0, tc.f1, p0, p1, n, HW / 4);
  else
    hipLaunchKernelGGL(pack_c4_pair_kernel, grid, dim3(kThreads), 0, st, tc.f0, tc.f1, p0, p1, n, HW);
  int rc = hip_check("pack_c4 (solve entry)");
  if (rc) return rc;
  tc.f0 = reinterpret_cast<const float*>(p0);
  tc.f1 = reinterpret_cast<const float*>(p1);
  dc.flags |= DPFT_FEATURES_C4;
  return DPFT_OK;
}

int solve_level_impl(const DpftLevelDesc* desc_in, const DpftLevelTensors* tensors_in, float* R, float* t,
                     float* jtj_out, float* jtr_out, void* ws, size_t ws_bytes, hipStream_t st) {
  int rc = check_desc(desc_in);
  if (rc) return rc;
  DpftLevelDesc dc = *desc_in;
  DpftLevelTensors tc = tensors_in ? *tensors_in : DpftLevelTensors{};
  if (tensors_in && packs_on_entry(dc) && (rc = pack_on_entry(*desc_in, dc, tc, ws, ws_bytes, st))) return rc;
  const DpftLevelDesc* desc = &dc;
  const DpftLevelTensors* tensors = tensors_in ? &tc : nullptr;
  for (int it = 0; it < desc->iters; ++it) {
    const bool last = it == desc->iters - 1;
    const int flags = (it == 0 ? DPFT_ITER_FIRST : 0) | ((it & 1) ? DPFT_ITER_REVERSE : 0);
    rc = iterate_impl(desc, tensors, R, t, last ? jtj_out : nullptr, last ? jtr_out : nullptr, nullptr, flags, ws,
                      ws_bytes, st);
    if (rc) return rc;
  }
  return DPFT_OK;
}

int sigma_extrema_impl(const DpftLevelDesc* descs, const DpftLevelTensors* tensors, int levels, void* workspace,
                       size_t workspace_bytes, hipStream_t st);

int pyramid_impl(const DpftLevelDesc* descs, const DpftLevelTensors* tt, int levels, float* R, float* t, void* ws,
                 size_t ws_bytes, hipStream_t st) {
  if (!descs || !tt || !R || !t || !ws) return fail(DPFT_E_INVALID, "null pointer");
  if (levels < 1 || levels > 8) return fail(DPFT_E_INVALID, "levels=%d outside [1, 8]", levels);
  int rc;
  for (int l = 0; l < levels; ++l) {
    if ((rc = check_desc(&descs[l]))) return rc;
    if ((rc = check_tensors(&tt[l], descs[l].flags))) return rc;
    if (ws_bytes < ws_need(descs[l])) return fail(DPFT_E_WORKSPACE, "workspace %zu < %zu", ws_bytes, ws_need(descs[l]));
    const DpftLevelDesc& a = descs[0];
    const DpftLevelDesc& d = descs[l];
    const uint32_t same = ~(DPFT_EXT_SLOT_MASK | DPFT_EXTREMA_READY | DPFT_SCHED_MASK);
    if (d.B != a.B || d.C != a.C || d.Cs != a.Cs || d.iters != a.iters || (d.flags & same) != (a.flags & same))
      return fail(DPFT_E_INVALID, "level %d: B / C / Cs / iters / flags differ from level 0 of the call", l);
    if ((d.flags & DPFT_REMOVE_TRU_SIGMA) && !(d.flags & DPFT_EXT_SLOT_MASK))
      return fail(DPFT_E_INVALID, "level %d: REMOVE_TRU_SIGMA needs DPFT_EXT_SLOT (one extrema pre-pass)", l);
  }
  // one pose-independent pre-pass for every level's sigma0 extrema, then the levels
  std::vector<DpftLevelDesc> d(descs, descs + levels);
  if (d[0].flags & DPFT_REMOVE_TRU_SIGMA) {
    if (levels > 4) return fail(DPFT_E_INVALID, "truncated sigma: at most 4 levels per pre-pass");
    for (auto& x : d) x.flags |= DPFT_EXTREMA_READY;
    if ((rc = sigma_extrema_impl(d.data(), tt, levels, ws, ws_bytes, st))) return rc;
  }
  for (int l = 0; l < levels; ++l)
    if ((rc = solve_level_impl(&d[l], &tt[l], R, t, nullptr, nullptr, ws, ws_bytes, st))) return rc;
  return DPFT_OK;
}

int residual_impl(const DpftLevelDesc* desc, const DpftLevelTensors* tt, int P, const float* R, const float* t,
                  float* loss, void* ws, size_t ws_bytes, hipStream_t st) {
  int rc = check_desc(desc);
  if (rc) return rc;
  if ((rc = check_tensors(tt, desc->flags))) return rc;
  if (!R || !t || !loss || !ws) return fail(DPFT_E_INVALID, "null pose / loss / workspace");
  if (P < 1 || P > kMaxPairs) return fail(DPFT_E_INVALID, "n_poses=%d outside [1, %d]", P, kMaxPairs);
  if (group_of(*desc) < desc->B) return fail(DPFT_E_INVALID, "DPFT_GROUP: solver entry points only");
  if (ws_bytes < ws_need_poses(*desc, P))
    return fail(DPFT_E_WORKSPACE, "workspace %zu < %zu", ws_bytes, ws_need_poses(*desc, P));
  const Geometry g = plan(*desc);
  if ((rc = launch_minmax(*desc, *tt, ws, st))) return rc;
  IterParams p = make_params(*desc, *tt, g, R, t, ws);
  p.fin.loss_out = loss;
  const dim3 grid(p.nblocks, P);
  const bool icp = (desc->flags & DPFT_COMBINE_ICP) != 0;
  if (desc->flags & DPFT_NO_UNCERTAINTY)
    hipLaunchKernelGGL((ic_residual_kernel<true, 2>), grid, dim3(kThreads), 0, st, p);
  else if (p.Cs == 1) {
    if (icp)
      hipLaunchKernelGGL((ic_residual_kernel<true, 1>), grid, dim3(kThreads), 0, st, p);
    else
      hipLaunchKernelGGL((ic_residual_kernel<true, 0>), grid, dim3(kThreads), 0, st, p);
  } else {
    if (icp)
      hipLaunchKernelGGL((ic_residual_kernel<false, 1>), grid, dim3(kThreads), 0, st, p);
    else
      hipLaunchKernelGGL((ic_residual_kernel<false, 0>), grid, dim3(kThreads), 0, st, p);
  }
  return hip_check("ic_residual_kernel");
}

}  // namespace

extern "C" {

size_t dpft_workspace_size(const DpftLevelDesc* desc) {
  if (check_desc(desc)) return 0;
  return ws_need(*desc);
}

int dpft_ic_iterate(const DpftLevelDesc* desc, const DpftLevelTensors* tensors, float* R, float* t, float* jtj_out,
                    float* jtr_out, int32_t* invalid_out, int first, void* workspace, size_t workspace_bytes,
                    void* hip_stream) {
  return iterate_impl(desc, tensors, R, t, jtj_out, jtr_out, invalid_out, first, workspace, workspace_bytes,
                      static_cast<hipStream_t>(hip_stream));
}

int dpft_ic_solve_level(const DpftLevelDesc* desc, const DpftLevelTensors* tensors, float* R, float* t,
                        float* jtj_out, float* jtr_out, void* workspace, size_t workspace_bytes, void* hip_stream) {
  return solve_level_impl(desc, tensors, R, t, jtj_out, jtr_out, workspace, workspace_bytes,
                          static_cast<hipStream_t>(hip_stream));
}

int dpft_ic_solve_pyramid(const DpftLevelDesc* descs, const DpftLevelTensors* tensors, int32_t levels, float* R,
                          float* t, void* workspace, size_t workspace_bytes, void* hip_stream) {
  return pyramid_impl(descs, tensors, levels, R, t, workspace, workspace_bytes, static_cast<hipStream_t>(hip_stream));
}

int dpft_ic_residual_level(const DpftLevelDesc* desc, const DpftLevelTensors* tt, const float* R, const float* t,
                           float* loss, void* ws, size_t ws_bytes, void* hip_stream) {
  return residual_impl(desc, tt, 1, R, t, loss, ws, ws_bytes, static_cast<hipStream_t>(hip_stream));
}

size_t dpft_residual_poses_workspace_size(const DpftLevelDesc* desc, int32_t n_poses) {
  if (check_desc(desc) || n_poses < 1 || n_poses > kMaxPairs) return 0;
  return ws_need_poses(*desc, n_poses);
}

int dpft_ic_residual_poses(const DpftLevelDesc* desc, const DpftLevelTensors* tt, int32_t n_poses, const float* R,
                           const float* t, float* loss, void* ws, size_t ws_bytes, void* hip_stream) {
  return residual_impl(desc, tt, n_poses, R, t, loss, ws, ws_bytes, static_cast<hipStream_t>(hip_stream));
}

int dpft_ic_reduce_only(const DpftLevelDesc* desc, const DpftLevelTensors* tt, const float* R, const float* t,
                        void* ws, size_t ws_bytes, void* hip_stream) {
  int rc = check_desc(desc);
  if (rc) return rc;
  if ((rc = check_tensors(tt, desc->flags))) return rc;
  if (ws_bytes < ws_core(*desc)) return fail(DPFT_E_WORKSPACE, "workspace %zu < %zu", ws_bytes, ws_core(*desc));
  const Geometry g = plan(*desc);
  return launch_reduce(make_params(*desc, *tt, g, R, t, ws), static_cast<hipStream_t>(hip_stream));
}

int dpft_ic_debug_pixels(const DpftLevelDesc* desc, const DpftLevelTensors* tt, const float* R, const float* t,
                         float* out, void* ws, size_t ws_bytes, void* hip_stream) {
  int rc = check_desc(desc);
  if (rc) return rc;
  if ((rc = check_tensors(tt, desc->flags))) return rc;
  if (!out || ws_bytes < ws_core(*desc)) return fail(DPFT_E_INVALID, "null output or small workspace");
  const Geometry g = plan(*desc);
  const IterParams p = make_params(*desc, *tt, g, R, t, ws);
  const int n = desc->B * desc->H * desc->W;
  hipLaunchKernelGGL(ic_debug_pixels_kernel, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0,
                     static_cast<hipStream_t>(hip_stream), p, out);
  return hip_check("ic_debug_pixels_kernel");
}

int dpft_ic_residual_map(const DpftLevelDesc* desc, const DpftLevelTensors* tt, const float* R, const float* t,
                         float* out, uint8_t* occ_out, void* ws, size_t ws_bytes, void* hip_stream) {
  int rc = check_desc(desc);
  if (rc) return rc;
  if ((rc = check_tensors(tt, desc->flags))) return rc;
  if (!(desc->flags & DPFT_NO_UNCERTAINTY))
    return fail(DPFT_E_INVALID, "the residual map is the IC tracker's (DPFT_NO_UNCERTAINTY)");
  if (!R || !t || !out || !ws || ws_bytes < ws_core(*desc)) return fail(DPFT_E_INVALID, "null pointer or small workspace");
  const Geometry g = plan(*desc);
  const IterParams p = make_params(*desc, *tt, g, R, t, ws);
  const long n = (long)desc->B * desc->H * desc->W;
  hipLaunchKernelGGL(ic_residual_map_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                     static_cast<hipStream_t>(hip_stream), p, out, occ_out);
  return hip_check("ic_residual_map_kernel");
}

int dpft_sigma_extrema_levels(const DpftLevelDesc* descs, const DpftLevelTensors* tensors, int32_t levels,
                              void* workspace, size_t workspace_bytes, void* hip_stream) {
  return sigma_extrema_impl(descs, tensors, levels, workspace, workspace_bytes, static_cast<hipStream_t>(hip_stream));
}
}  // extern "C"

namespace {
int sigma_extrema_impl(const DpftLevelDesc* descs, const DpftLevelTensors* tensors, int levels, void* workspace,
                       size_t workspace_bytes, hipStream_t st) {
  if (!descs || !tensors || !workspace) return fail(DPFT_E_INVALID, "null pointer");
  if (levels < 1 || levels > 4) return fail(DPFT_E_INVALID, "levels=%d outside [1, 4]", levels);
  MMLevels a;
  a.groups = 1;
  size_t nmax = 0;
  for (int l = 0; l < 4; ++l) {
    a.s[l] = nullptr;
    a.n[l] = 0;
    a.slot[l] = 0;
  }
  for (int l = 0; l < levels; ++l) {
    const DpftLevelDesc& d = descs[l];
    int rc = check_desc(&d);
    if (rc) return rc;
    const int xslot = (int)((d.flags & DPFT_EXT_SLOT_MASK) >> DPFT_EXT_SLOT_SHIFT);
    if (!xslot) return fail(DPFT_E_INVALID, "level %d has no extrema slot (DPFT_EXT_SLOT)", l);
    if (!tensors[l].s0) return fail(DPFT_E_INVALID, "level %d: null sigma0", l);
    if (workspace_bytes < ws_core(d)) return fail(DPFT_E_WORKSPACE, "workspace %zu < %zu", workspace_bytes, ws_core(d));
    if (l == 0) a.groups = d.B / group_of(d);
    if (d.B / group_of(d) != a.groups) return fail(DPFT_E_INVALID, "level %d: another DPFT_GROUP than level 0", l);
    a.s[l] = tensors[l].s0;
    a.n[l] = (size_t)group_of(d) * d.Cs * d.H * d.W;  // per batch
    a.slot[l] = ext_word(d);
    nmax = std::max(nmax, a.n[l]);
  }
  // partial extrema: 2 words per workgroup and (level, batch), kMaxMMBlocks pairs in all
  const int grid = (int)std::max<size_t>(1, std::min<size_t>(std::min<size_t>((nmax + kThreads * 16 - 1) / (kThreads * 16), kMMGrid),
                                                              (size_t)kMaxMMBlocks / ((size_t)levels * a.groups)));
  static_assert(4 * 2 * kMMGrid <= 2 * kMaxMMBlocks, "per-level minmax partials");
  hipLaunchKernelGGL(minmax_levels_kernel, dim3(grid, levels * a.groups), dim3(kThreads), 0, st, a,
                     static_cast<uint32_t*>(workspace));
  return hip_check("minmax_levels_kernel");
}
// ---------------------------------------------------------------------------------
// Jacobian API, materialised (the reference's solver methods precompute_jacobian_
// components / compose_inverse_jacobians / compute_jtj / compute_jtr, algorithms.py:
// 812-887): not on the solve path, which never writes J.  Elementwise kernels plus a
// two-stage fixed-order fp64 reduction.

// unit-normalised 3x3 Sobel with replicate padding (feature_gradient, 1844-1865):
// f [P planes of H x W] -> g [P][2][H][W]
__global__ __launch_bounds__(kThreads) void feature_gradient_kernel(const float* __restrict__ f, float* g, long P,
                                                                    int H, int W) {
  const long i = (long)blockIdx.x * kThreads + threadIdx.x;
  const long HW = (long)H * W;
  if (i >= P * HW) return;
  const long pl = i / HW;
  const int rem = (int)(i - pl * HW), y = rem / W, x = rem - y * W;
  const float* F = f + pl * HW;
  const int ym = max(y - 1, 0), yp = min(y + 1, H - 1), xm = max(x - 1, 0), xp = min(x + 1, W - 1);
  auto at = [&](int yy, int xx) { return F[(long)yy * W + xx]; };
  const float dx = ((at(ym, xp) - at(ym, xm)) + 2.0f * (at(y, xp) - at(y, xm))) + (at(yp, xp) - at(yp, xm));
  const float dy = ((at(yp, xm) - at(ym, xm)) + 2.0f * (at(yp, x) - at(ym, x))) + (at(yp, xp) - at(ym, xp));
  const float mag = sqrtf(dx * dx + dy * dy + 1e-8f);
  g[pl * 2 * HW + rem] = dx / mag;
  g[(pl * 2 + 1) * HW + rem] = dy / mag;
}

// compute_jacobian_warping (1884-1917) at the origin: Jx, Jy [B][HW][6]
__global__ __launch_bounds__(kThreads) void warp_jacobian_kernel(const float* __restrict__ invD0,
                                                                 const float* __restrict__ K,
                                                                 const float* __restrict__ px,
                                                                 const float* __restrict__ py, float* Jx, float* Jy,
                                                                 int B, long HW) {
  const long i = (long)blockIdx.x * kThreads + threadIdx.x;
  if (i >= (long)B * HW) return;
  const int b = (int)(i / HW);
  const float x = px[i], y = py[i], d = invD0[i], fx = K[4 * b], fy = K[4 * b + 1], xy = x * y;
  const float jx[6] = {-xy, 1.0f + x * x, -y, d, 0.0f, -d * x};
  const float jy[6] = {-1.0f - y * y, xy, x, 0.0f, d, -d * y};
  for (int k = 0; k < 6; ++k) {
    Jx[6 * i + k] = jx[k] * fx;
    Jy[6 * i + k] = jy[k] * fy;
  }
}

// compose_inverse_jacobians (867-887) + compute_jacobian_dIdp (1867-1882):
// a = -gx / s - r (s0 hx / s^3), b likewise, J = -(a Jx + b Jy) -> J [B][C][HW][6].
// sigma0 / grad_sigma0 carry Cs = 1 or C channels.
__global__ __launch_bounds__(kThreads) void inverse_jacobian_kernel(
    const float* __restrict__ res, const float* __restrict__ sigma, const float* __restrict__ s0,
    const float* __restrict__ gf0, const float* __restrict__ gs0, const float* __restrict__ Jx,
    const float* __restrict__ Jy, float* J, int B, int C, int Cs, long HW) {
  const long i = (long)blockIdx.x * kThreads + threadIdx.x;
  if (i >= (long)B * C * HW) return;
  const long bc = i / HW, p = i - bc * HW;
  const int b = (int)(bc / C), c = (int)(bc - (long)b * C), cs = Cs == 1 ? 0 : c;
  const long bs = (long)b * Cs + cs;
  const float r = res[i], s = sigma[i], sz = s0[bs * HW + p];
  const float s3 = (s * s) * s;
  const float a = -gf0[(bc * 2) * HW + p] / s - r * ((sz * gs0[(bs * 2) * HW + p]) / s3);
  const float bb = -gf0[(bc * 2 + 1) * HW + p] / s - r * ((sz * gs0[(bs * 2 + 1) * HW + p]) / s3);
  const float* jx = Jx + ((long)b * HW + p) * 6;
  const float* jy = Jy + ((long)b * HW + p) * 6;
  for (int k = 0; k < 6; ++k) J[6 * i + k] = -(a * jx[k] + bb * jy[k]);
}

// J^T J, J^T r over n rows of 6 per pair: stage 1, block k of pair b sums rows
// [n k / nb, n (k+1) / nb) into 27 fp64 partials (fixed order: thread-strided, then a
// fixed tree); stage 2 sums a pair's nb partials in order.
constexpr int kJtjBlocks = 128;
__global__ __launch_bounds__(kThreads) void jtj_partial_kernel(const float* __restrict__ J,
                                                               const float* __restrict__ r, long n, double* part) {
  const int b = blockIdx.y, k = blockIdx.x, nb = gridDim.x;
  const long beg = n * k / nb, end = n * (k + 1) / nb;
  double acc[27];
#pragma unroll
  for (int q = 0; q < 27; ++q) acc[q] = 0.0;
  const float* Jb = J + (size_t)b * n * 6;
  const float* rb = r ? r + (size_t)b * n : nullptr;
  for (long row = beg + threadIdx.x; row < end; row += kThreads) {
    double j[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) j[q] = Jb[6 * row + q];
    int m = 0;
#pragma unroll
    for (int u = 0; u < 6; ++u)
#pragma unroll
      for (int v = u; v < 6; ++v) acc[m++] += j[u] * j[v];
    if (rb) {
      const double rr = rb[row];
#pragma unroll
      for (int u = 0; u < 6; ++u) acc[21 + u] += j[u] * rr;
    }
  }
  __shared__ double sm[kThreads];
#pragma unroll
  for (int q = 0; q < 27; ++q) {
    sm[threadIdx.x] = acc[q];
    __syncthreads();
    for (int w = kThreads / 2; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) sm[threadIdx.x] += sm[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) part[((size_t)b * nb + k) * 27 + q] = sm[0];
    __syncthreads();
  }
}

__global__ __launch_bounds__(64) void jtj_final_kernel(const double* __restrict__ part, int nb, float* jtj,
                                                       float* jtr) {
  const int b = blockIdx.x, q = threadIdx.x;
  if (q >= 27) return;
  double s = 0.0;
  for (int k = 0; k < nb; ++k) s += part[((size_t)b * nb + k) * 27 + q];
  if (q < 21) {
    int u = 0, m = q;
    while (m >= 6 - u) {
      m -= 6 - u;
      ++u;
    }
    const int v = u + m;
    jtj[36 * b + 6 * u + v] = (float)s;
    jtj[36 * b + 6 * v + u] = (float)s;
  } else if (jtr) {
    jtr[6 * b + q - 21] = (float)s;
  }
}

// One thread per (sample s, pair b): H = JtJ_b + diag(diag_add[s, b]) + 1e-6 tr(JtJ_b) I,
// xi = H^-1 JtR_b (fp64 Cholesky), pose_out[s, b] = the inverse-compositional update of
// pose_b (dpft_ic_damped_update).
__global__ __launch_bounds__(kThreads) void damped_update_kernel(const float* __restrict__ jtj,
                                                                 const float* __restrict__ jtr,
                                                                 const float* __restrict__ diag_add, int S, int B,
                                                                 const float* __restrict__ R,
                                                                 const float* __restrict__ t, float* R_out,
                                                                 float* t_out) {
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= S * B) return;
  const int b = i % B;
  double ju[21], jr[6], dg[6];
  int k = 0;
  for (int r = 0; r < 6; ++r)
    for (int c = r; c < 6; ++c) ju[k++] = jtj[36 * b + 6 * r + c];
  for (int r = 0; r < 6; ++r) {
    jr[r] = jtr[6 * b + r];
    dg[r] = diag_add ? diag_add[6 * i + r] : 0.0;
  }
  float* Ro = R_out + 9 * (size_t)i;
  float* to = t_out + 3 * (size_t)i;
  for (int r = 0; r < 9; ++r) Ro[r] = R[9 * b + r];
  for (int r = 0; r < 3; ++r) to[r] = t[3 * b + r];
  solve_and_update(ju, jr, Ro, to, dg);
}

// Diagnostic streaming read (dpft_read_probe): every 16-byte word of a buffer once,
// kProbeDepth loads in flight per lane, one float per wave written.  The measured HBM read
// ceiling bench.py reports beside the roofline's spec peak.
constexpr int kProbeGrid = DPFT_PROBE_GRID;    // 16 workgroups per CU
constexpr int kProbeDepth = DPFT_PROBE_DEPTH;  // 16-byte loads in flight per lane
// Streaming copies for the measured copy ceiling (read + write bytes / time).  Mode 0: the
// plain float4 copy of MI355X_MICROARCH.md's bandwidth table (one 16-byte element per thread);
// mode 1: grid-stride, 16-byte non-temporal loads and stores, kProbeDepth in flight per lane.
__global__ __launch_bounds__(kThreads) void copy_probe_flat_kernel(const f32x4* __restrict__ src,
                                                                   f32x4* __restrict__ dst, size_t n4) {
  const size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < n4) dst[i] = src[i];
}
__global__ __launch_bounds__(kThreads) void copy_probe_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst,
                                                              size_t n4) {
  const size_t stride = (size_t)gridDim.x * kThreads;
  size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x;
  for (; i + (kProbeDepth - 1) * stride < n4; i += kProbeDepth * stride) {
    f32x4 v[kProbeDepth];
#pragma unroll
    for (int k = 0; k < kProbeDepth; ++k) v[k] = __builtin_nontemporal_load(src + i + k * stride);
#pragma unroll
    for (int k = 0; k < kProbeDepth; ++k) __builtin_nontemporal_store(v[k], dst + i + k * stride);
  }
  for (; i < n4; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

template <bool NT>
__global__ __launch_bounds__(kThreads) void read_probe_kernel(const f32x4* __restrict__ p, size_t n4, float* out) {
  const size_t stride = (size_t)gridDim.x * kThreads;
  size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x;
  auto ld = [&](size_t k) { return NT ? __builtin_nontemporal_load(p + k) : p[k]; };
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (; i + (kProbeDepth - 1) * stride < n4; i += kProbeDepth * stride) {
    f32x4 v[kProbeDepth];
#pragma unroll
    for (int k = 0; k < kProbeDepth; ++k) v[k] = ld(i + k * stride);
#pragma unroll
    for (int k = 0; k < kProbeDepth; ++k) acc += v[k];
  }
  for (; i < n4; i += stride) acc += ld(i);
  float v = (acc.x + acc.y) + (acc.z + acc.w);
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6)] = v;
}

// Encoder block epilogue in eval mode (submodules.py convLayer: BatchNorm2d with running
// statistics, then ELU(alpha = 1)): y = x * a_c + b_c with a = w / sqrt(var + eps),
// b = bias - mean * a (the linear form ATen's CPU inference applies), then
// y > 0 ? y : expm1(y), in place, one 16-byte read and write per four values (two
// elementwise passes in the torch modules).  chan = [a | b], C floats each.  NHWC: the
// four values of a 16-byte unit are channels c .. c + 3 (C % 4 == 0); NCHW: one channel
// (H W % 4 == 0).
__device__ inline float elu1(float y) { return y > 0.0f ? y : expm1f(y); }
__device__ inline float bn_elu1(float x, const float* __restrict__ chan, uint32_t C, uint32_t c) {
  return elu1(x * chan[c] + chan[C + c]);
}
// The batchnorm scale / shift of channels c .. c + 3 (c % 4 == 0): two 16-byte loads when
// `chan` is 16-byte aligned (CV) instead of eight 4-byte ones -- per 16-byte unit of
// features the 4-byte loads were 8 of the kernel's 10 memory instructions (dpft_bn_elu_pack:
// 3.9 -> 6.1 TB/s, bench.py encoder leg)
template <bool CV>
__device__ inline f32x4 bn_elu4(f32x4 v, const float* __restrict__ chan, uint32_t C, uint32_t c) {
  f32x4 a, sh;
  if constexpr (CV) {
    a = *reinterpret_cast<const f32x4*>(chan + c);
    sh = *reinterpret_cast<const f32x4*>(chan + C + c);
  } else {
    a = f32x4{chan[c], chan[c + 1], chan[c + 2], chan[c + 3]};
    sh = f32x4{chan[C + c], chan[C + c + 1], chan[C + c + 2], chan[C + c + 3]};
  }
  return f32x4{elu1(v.x * a.x + sh.x), elu1(v.y * a.y + sh.y), elu1(v.z * a.z + sh.z), elu1(v.w * a.w + sh.w)};
}
template <bool NHWC, bool CV>
__global__ __launch_bounds__(kThreads) void bn_elu_kernel(f32x4* __restrict__ x, const float* __restrict__ chan,
                                                          uint32_t n4, uint32_t C, uint32_t inner4) {
  const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= n4) return;
  f32x4 v = __builtin_nontemporal_load(x + i);
  if (NHWC) {
    v = bn_elu4<CV>(v, chan, C, (i % (C / 4)) * 4);
  } else {
    const uint32_t c = (i / inner4) % C;
    v.x = bn_elu1(v.x, chan, C, c);
    v.y = bn_elu1(v.y, chan, C, c);
    v.z = bn_elu1(v.z, chan, C, c);
    v.w = bn_elu1(v.w, chan, C, c);
  }
  __builtin_nontemporal_store(v, x + i);
}

// dpft_bn_elu_pack: bn_elu_kernel<true>'s epilogue on a channels_last conv output, stored to
// the channel-quad layout with pack_c4_nhwc_kernel's mapping (thread r of pair row b =
// blockIdx.y reads quad r of the pair's [HW][C] block; 64 lanes = 64 / Q pixels x Q planes,
// one 128-byte run per plane at Q = 8).  The conv output is read once (non-temporal).
template <bool CV>
__global__ __launch_bounds__(kThreads) void bn_elu_pack_kernel(const f32x4* __restrict__ src,
                                                               const float* __restrict__ chan,
                                                               f32x4* __restrict__ dst, uint32_t n, uint32_t Q,
                                                               uint32_t HW) {
  const uint32_t r = blockIdx.x * kThreads + threadIdx.x;
  if (r >= n) return;
  const size_t base = (size_t)blockIdx.y * n;
  const uint32_t pix = r / Q, q = r - pix * Q, C = 4 * Q, c = 4 * q;
  const f32x4 v = bn_elu4<CV>(__builtin_nontemporal_load(src + base + r), chan, C, c);
  dst[base + (size_t)q * HW + pix] = v;
}
}  // namespace

extern "C" {

int dpft_feature_gradient(const float* f, float* grad, int32_t B, int32_t C, int32_t H, int32_t W,
                          void* hip_stream) {
  if (!f || !grad || f == grad) return fail(DPFT_E_INVALID, "null or aliased pointer");
  if (B < 1 || C < 1 || H < 1 || W < 1) return fail(DPFT_E_INVALID, "bad shape B=%d C=%d H=%d W=%d", B, C, H, W);
  const long n = (long)B * C * H * W;
  hipLaunchKernelGGL(feature_gradient_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                     static_cast<hipStream_t>(hip_stream), f, grad, (long)B * C, H, W);
  return hip_check("feature_gradient_kernel");
}

int dpft_warp_jacobian(const float* invD0, const float* K, const float* px, const float* py, float* Jx, float* Jy,
                       int32_t B, int32_t H, int32_t W, void* hip_stream) {
  if (!invD0 || !K || !px || !py || !Jx || !Jy) return fail(DPFT_E_INVALID, "null pointer");
  if (B < 1 || H < 1 || W < 1) return fail(DPFT_E_INVALID, "bad shape B=%d H=%d W=%d", B, H, W);
  const long n = (long)B * H * W;
  hipLaunchKernelGGL(warp_jacobian_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                     static_cast<hipStream_t>(hip_stream), invD0, K, px, py, Jx, Jy, B, (long)H * W);
  return hip_check("warp_jacobian_kernel");
}

int dpft_inverse_jacobian(const float* res, const float* sigma, const float* sigma0, const float* grad_f0,
                          const float* grad_sigma0, const float* Jx, const float* Jy, float* J, int32_t B, int32_t C,
                          int32_t Cs, int32_t H, int32_t W, void* hip_stream) {
  if (!res || !sigma || !sigma0 || !grad_f0 || !grad_sigma0 || !Jx || !Jy || !J)
    return fail(DPFT_E_INVALID, "null pointer");
  if (B < 1 || C < 1 || H < 1 || W < 1 || (Cs != 1 && Cs != C))
    return fail(DPFT_E_INVALID, "bad shape B=%d C=%d Cs=%d H=%d W=%d", B, C, Cs, H, W);
  const long n = (long)B * C * H * W;
  hipLaunchKernelGGL(inverse_jacobian_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                     static_cast<hipStream_t>(hip_stream), res, sigma, sigma0, grad_f0, grad_sigma0, Jx, Jy, J, B, C,
                     Cs, (long)H * W);
  return hip_check("inverse_jacobian_kernel");
}

size_t dpft_normal_equations_workspace_size(int32_t B) { return (size_t)std::max(B, 0) * kJtjBlocks * 27 * sizeof(double); }

int dpft_normal_equations(const float* J, const float* r, int64_t n, int32_t B, float* jtj, float* jtr, void* ws,
                          size_t ws_bytes, void* hip_stream) {
  if (!J || !jtj || !ws) return fail(DPFT_E_INVALID, "null pointer");
  if (B < 1 || n < 1) return fail(DPFT_E_INVALID, "bad shape B=%d n=%lld", B, (long long)n);
  if (ws_bytes < dpft_normal_equations_workspace_size(B))
    return fail(DPFT_E_WORKSPACE, "workspace %zu < %zu", ws_bytes, dpft_normal_equations_workspace_size(B));
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(jtj_partial_kernel, dim3(kJtjBlocks, B), dim3(kThreads), 0, st, J, r, (long)n, part);
  int rc = hip_check("jtj_partial_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(jtj_final_kernel, dim3(B), dim3(64), 0, st, part, kJtjBlocks, jtj, r ? jtr : nullptr);
  return hip_check("jtj_final_kernel");
}

int dpft_ic_damped_update(const float* jtj, const float* jtr, const float* diag_add, int32_t S, int32_t B,
                          const float* R, const float* t, float* R_out, float* t_out, void* hip_stream) {
  if (!jtj || !jtr || !R || !t || !R_out || !t_out) return fail(DPFT_E_INVALID, "null pointer");
  if (S < 1 || B < 1 || (long)S * B > (1L << 24)) return fail(DPFT_E_INVALID, "bad S=%d B=%d", S, B);
  const int n = S * B;
  hipLaunchKernelGGL(damped_update_kernel, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0,
                     static_cast<hipStream_t>(hip_stream), jtj, jtr, diag_add, S, B, R, t, R_out, t_out);
  return hip_check("damped_update_kernel");
}

size_t dpft_read_probe_out_floats(void) { return (size_t)kProbeGrid * (kThreads / 64); }

int dpft_copy_probe(const void* src, void* dst, size_t bytes, int32_t mode, void* hip_stream) {
  if (!src || !dst) return fail(DPFT_E_INVALID, "null pointer");
  if (bytes < 16 || ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15))
    return fail(DPFT_E_INVALID, "need >= 16 bytes, 16-byte aligned");
  const size_t n4 = bytes / 16;
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  const f32x4* s4 = static_cast<const f32x4*>(src);
  f32x4* d4 = static_cast<f32x4*>(dst);
  if (mode == 0) {
    if (n4 > (size_t)kThreads * 0x7fffffffu) return fail(DPFT_E_INVALID, "copy too large for one flat launch");
    hipLaunchKernelGGL(copy_probe_flat_kernel, dim3((unsigned)((n4 + kThreads - 1) / kThreads)), dim3(kThreads), 0, st,
                       s4, d4, n4);
  } else {
    hipLaunchKernelGGL(copy_probe_kernel, dim3(kProbeGrid), dim3(kThreads), 0, st, s4, d4, n4);
  }
  return hip_check("copy_probe_kernel");
}

int dpft_read_probe(const void* buf, size_t bytes, int32_t nontemporal, float* out, void* hip_stream) {
  if (!buf || !out) return fail(DPFT_E_INVALID, "null pointer");
  if (bytes < 16 || (reinterpret_cast<uintptr_t>(buf) & 15)) return fail(DPFT_E_INVALID, "need >= 16 aligned bytes");
  const f32x4* p = static_cast<const f32x4*>(buf);
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  if (nontemporal)
    hipLaunchKernelGGL(read_probe_kernel<true>, dim3(kProbeGrid), dim3(kThreads), 0, st, p, bytes / 16, out);
  else
    hipLaunchKernelGGL(read_probe_kernel<false>, dim3(kProbeGrid), dim3(kThreads), 0, st, p, bytes / 16, out);
  return hip_check("read_probe_kernel");
}

size_t dpft_preprocess_workspace_size(void) { return kCtrlBytes; }

int dpft_preprocess_depth(const float* depth, int32_t B, int32_t H, int32_t W, int32_t levels, float* const* invd_out,
                          float* const* depth_out, void* ws, size_t ws_bytes, void* hip_stream) {
  if (!depth || !invd_out || !ws) return fail(DPFT_E_INVALID, "null pointer");
  if (B < 1 || H < 1 || W < 1 || levels < 1 || levels > 4 || (H >> (levels - 1)) < 1 || (W >> (levels - 1)) < 1)
    return fail(DPFT_E_INVALID, "bad shape B=%d H=%d W=%d levels=%d", B, H, W, levels);
  if (ws_bytes < kCtrlBytes) return fail(DPFT_E_WORKSPACE, "workspace %zu < %zu", ws_bytes, kCtrlBytes);
  PyrOut out;
  for (int l = 0; l < 4; ++l) {
    out.invd[l] = l < levels ? invd_out[l] : nullptr;
    out.depth[l] = (l < levels && depth_out) ? depth_out[l] : nullptr;
    if (l < levels && !out.invd[l]) return fail(DPFT_E_INVALID, "null invD output of level %d", l);
  }
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  uint32_t* ctrl = static_cast<uint32_t*>(ws);
  const size_t n = (size_t)B * H * W;
  const int grid = (int)std::min<size_t>((n + kThreads * 16 - 1) / (kThreads * 16), kMaxMMBlocks);
  hipLaunchKernelGGL(invd_minmax_kernel, dim3(grid), dim3(kThreads), 0, st, depth, n, ctrl);
  int rc = hip_check("invd_minmax_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(invd_pyramid_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads), levels), dim3(kThreads), 0,
                     st, depth, B, H, W, ctrl, out);
  return hip_check("invd_pyramid_kernel");
}

int dpft_pack_features(const float* src, float* dst, int32_t B, int32_t C, int32_t H, int32_t W, void* hip_stream) {
  if (!src || !dst || src == dst) return fail(DPFT_E_INVALID, "null or aliased pointer");
  if (B < 1 || C < 4 || C % 4 != 0 || H < 1 || W < 1 || (long)H * W >= (1L << 30))
    return fail(DPFT_E_INVALID, "bad shape B=%d C=%d H=%d W=%d (C %% 4 == 0 needed)", B, C, H, W);
  const long n = (long)B * (C / 4) * H * W;
  hipLaunchKernelGGL(pack_c4_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                     static_cast<hipStream_t>(hip_stream), src, reinterpret_cast<f32x4*>(dst), n, H * W);
  return hip_check("pack_c4_kernel");
}

int dpft_pack_features_nhwc(const float* src, float* dst, int32_t B, int32_t C, int32_t H, int32_t W,
                            void* hip_stream) {
  if (!src || !dst || src == dst) return fail(DPFT_E_INVALID, "null or aliased pointer");
  if (B < 1 || B > 65535 || C < 4 || C % 4 != 0 || H < 1 || W < 1 || (long)H * W * (C / 4) >= (1L << 31))
    return fail(DPFT_E_INVALID, "bad shape B=%d C=%d H=%d W=%d (C %% 4 == 0 needed)", B, C, H, W);
  if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15)
    return fail(DPFT_E_INVALID, "src / dst must be 16-byte aligned");
  const uint32_t Q = (uint32_t)(C / 4), HW = (uint32_t)H * (uint32_t)W, n = HW * Q;
  hipLaunchKernelGGL(pack_c4_nhwc_kernel, dim3((n + kThreads - 1) / kThreads, (unsigned)B), dim3(kThreads), 0,
                     static_cast<hipStream_t>(hip_stream), reinterpret_cast<const f32x4*>(src),
                     reinterpret_cast<f32x4*>(dst), n, Q, HW);
  return hip_check("pack_c4_nhwc_kernel");
}

int dpft_bn_elu(float* x, const float* chan, int64_t n, int32_t C, int64_t inner, int32_t nhwc, void* hip_stream) {
  if (!x || !chan) return fail(DPFT_E_INVALID, "null pointer");
  if (n < 4 || C < 1 || inner < 1 || n % 4 != 0 || n / 4 >= (1L << 32) - kThreads || n % (C * inner) != 0)
    return fail(DPFT_E_INVALID, "bad size n=%ld C=%d inner=%ld", (long)n, C, (long)inner);
  if (reinterpret_cast<uintptr_t>(x) & 15) return fail(DPFT_E_INVALID, "x must be 16-byte aligned");
  if (nhwc ? (C % 4 != 0 || inner != 1) : (inner % 4 != 0))
    return fail(DPFT_E_INVALID, "the 16-byte units must not straddle channels (C=%d inner=%ld)", C, (long)inner);
  const uint32_t n4 = (uint32_t)(n / 4);
  const dim3 grid((n4 + kThreads - 1) / kThreads);
  const hipStream_t st = static_cast<hipStream_t>(hip_stream);
  f32x4* x4 = reinterpret_cast<f32x4*>(x);
  const bool cv = (reinterpret_cast<uintptr_t>(chan) & 15) == 0;
  if (nhwc && cv)
    hipLaunchKernelGGL((bn_elu_kernel<true, true>), grid, dim3(kThreads), 0, st, x4, chan, n4, (uint32_t)C, 1u);
  else if (nhwc)
    hipLaunchKernelGGL((bn_elu_kernel<true, false>), grid, dim3(kThreads), 0, st, x4, chan, n4, (uint32_t)C, 1u);
  else
    hipLaunchKernelGGL((bn_elu_kernel<false, false>), grid, dim3(kThreads), 0, st, x4, chan, n4, (uint32_t)C,
                       (uint32_t)(inner / 4));
  return hip_check("bn_elu_kernel");
}

int dpft_bn_elu_pack(const float* x, const float* chan, float* out, int32_t B, int32_t C, int32_t H, int32_t W,
                     void* hip_stream) {
  if (!x || !chan || !out || x == out) return fail(DPFT_E_INVALID, "null or aliased pointer");
  if (B < 1 || B > 65535 || C < 4 || C % 4 != 0 || H < 1 || W < 1 || (long)H * W * (C / 4) >= (1L << 31))
    return fail(DPFT_E_INVALID, "bad shape B=%d C=%d H=%d W=%d (C %% 4 == 0 needed)", B, C, H, W);
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) & 15)
    return fail(DPFT_E_INVALID, "x / out must be 16-byte aligned");
  const uint32_t Q = (uint32_t)(C / 4), HW = (uint32_t)H * (uint32_t)W, n = HW * Q;
  const dim3 grid((n + kThreads - 1) / kThreads, (unsigned)B);
  const hipStream_t st = static_cast<hipStream_t>(hip_stream);
  if ((reinterpret_cast<uintptr_t>(chan) & 15) == 0)
    hipLaunchKernelGGL(bn_elu_pack_kernel<true>, grid, dim3(kThreads), 0, st, reinterpret_cast<const f32x4*>(x), chan,
                       reinterpret_cast<f32x4*>(out), n, Q, HW);
  else
    hipLaunchKernelGGL(bn_elu_pack_kernel<false>, grid, dim3(kThreads), 0, st, reinterpret_cast<const f32x4*>(x),
                       chan, reinterpret_cast<f32x4*>(out), n, Q, HW);
  return hip_check("bn_elu_pack_kernel");
}

int dpft_version(void) { return DPFT_ABI_VERSION; }

const char* dpft_last_error(void) { return g_err; }

}  // extern "C"
