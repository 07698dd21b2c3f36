/*
 * dpft_ic.h -- C ABI of libdpft_ic.so, the MI355X (gfx950) implementation of the
 * trust-region inverse-compositional (U_IC) solver hot path of
 * Deep Probabilistic Feature-metric Tracking.
 *
 * Plain pointers and sizes only; every device pointer is caller-owned (torch
 * caching allocator or hipMalloc).  The library never allocates, never
 * synchronises the stream, and enqueues all work on the caller's stream, so
 * every entry point can be captured into a hipGraph.
 *
 * Reference interfaces replaced (paths relative to the reference repo):
 *   dpft_ic_solve_level    <- TrustRegionInverseWUncertainty.forward
 *                             code/models/algorithms.py:611-723
 *                             (+ precompute_jacobian_components 848-865,
 *                                compute_inverse_residuals 1992-2015,
 *                                compose_residuals 1960-1989,
 *                                compose_inverse_jacobians 867-887,
 *                                compute_jtj / compute_jtr 812-834,
 *                                GN_solver -> lev_mar_H -> inverse_update_pose
 *                                836-846, 2094-2103, 2035-2054)
 *   dpft_ic_solve_pyramid  <- the coarse-to-fine level loop of LeastSquareTracking.forward
 *                             code/models/LeastSquareTracking.py:349-445 (tr_update3..0)
 *   dpft_ic_iterate        <- ONE pass of the loop body algorithms.py:646-693
 *   dpft_ic_residual_map   <- compute_warped_residual algorithms.py:1919-1957 (IC tracker)
 *   dpft_ic_residual_level <- TrustRegionInverseWUncertainty.forward_residuals
 *                             algorithms.py:725-786 (+ compute_avg_loss 2119-2137)
 *   dpft_workspace_size / dpft_version / dpft_last_error: library plumbing.
 *
 * Semantics follow the reference exactly where they are observable:
 *   - K is per pair [B,4] = (fx, fy, cx, cy) already divided by 2^level
 *     (LeastSquareTracking.py:350: `K >> l` on a float tensor = K / 2^l);
 *   - the truncated-sigma and invalid-normal masks use min / max over the whole
 *     batch passed in one call (algorithms.py:1975-1980, 2168);
 *   - the Jacobian is not masked; invalid pixels only get a weighted residual of
 *     1e-6 (algorithms.py:867-887, 1982-1983);
 *   - exactly `iters` Gauss-Newton steps, no early exit (algorithms.py:646);
 *   - pose update R <- R Exp(-w), t <- R (-Exp(-w) v) + t (algorithms.py:2035-2054).
 *
 * Return codes: DPFT_OK, or a negative DPFT_E_* code; dpft_last_error() gives a
 * thread-local message.  Non-finite Jacobians / residuals (the reference's
 * `assert check_nan(...) == 0`, algorithms.py:886, 1988) are reported through
 * the device status word (DPFT_STATUS_NONFINITE), read by the caller once per
 * solve.
 */
#ifndef DPFT_IC_H
#define DPFT_IC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPFT_ABI_VERSION 2

/* flags of DpftLevelDesc */
#define DPFT_REMOVE_TRU_SIGMA 0x1u /* --remove_tru_sigma (algorithms.py:1975-1980) */
#define DPFT_COMBINE_ICP      0x2u /* --combine_ICP (algorithms.py:668-689)        */
#define DPFT_NO_UNCERTAINTY   0x4u /* IC tracker, TrustRegionBase (algorithms.py:23-139):
                                      sigma = 1, s0/s1 ignored (may be NULL), occluded
                                      residual 1e-3; excludes the two flags above     */
#define DPFT_FEATURES_C4      0x8u /* f0 / f1 in channel-quad layout [B][C/4][H][W][4]
                                      (dpft_pack_features); needs C % 4 == 0 and Cs == 1
                                      (or NO_UNCERTAINTY).  Same values, coalesced
                                      16-byte loads of 4 channels per pixel / tap.    */

/* Channel-quad reduce schedule (bits 4-5; FEATURES_C4 with C = 16 or 32 only, else
   ignored).  AUTO picks per level; the others force one kernel -- same arithmetic,
   a different summation grouping -- for tests and tuning:
     MARCH   a wave walks a band of rows of one 62-column strip with a window of f0 rows
     SPLIT   a workgroup per (strip, row), the 4 waves split the channel quads
             (AUTO: levels of at most 40000 pixels per pair) */
#define DPFT_SCHED_MASK    0x30u
#define DPFT_SCHED_AUTO    0x00u
#define DPFT_SCHED_MARCH   0x10u
#define DPFT_SCHED_SPLIT   0x20u

/* Per-level sigma0 extrema slots (pyramid solves, one pre-pass for all levels):
 * DPFT_EXT_SLOT(k) (k = 0..7) keeps this level's extrema in workspace slot k;
 * DPFT_EXTREMA_READY: dpft_sigma_extrema_levels already filled the slot, so the
 * first iteration of the level does not recompute them.                          */
#define DPFT_EXT_SLOT_SHIFT 12
#define DPFT_EXT_SLOT_MASK  0xF000u
#define DPFT_EXT_SLOT(k)    ((((uint32_t)(k)) + 1u) << DPFT_EXT_SLOT_SHIFT)
#define DPFT_EXTREMA_READY  0x10000u

/* Independent batches in one call (bits 20-31): DPFT_GROUP(n) splits the B pairs into
 * B / n consecutive batches of n pairs (B % n == 0, at most 32 batches), each solved
 * exactly as a call of its own -- its own batch-global truncated-sigma extrema
 * (algorithms.py:1975-1980) and sigma0 pre-pass -- while every launch covers all B
 * pairs (fewer, larger launches: the per-launch ramp, finish spread and finalize are
 * paid once for all batches).  With COMBINE_ICP each batch also keeps its own depth1
 * extrema (the normal map's invalid-depth test, algorithms.py:2168).  0 (or n >= B): the
 * call is one batch.  Solver entry points only (the residual entry points reject it). */
#define DPFT_GROUP_SHIFT 20
#define DPFT_GROUP_MASK  0xFFF00000u
#define DPFT_GROUP(n)    ((((uint32_t)(n)) << DPFT_GROUP_SHIFT) & DPFT_GROUP_MASK)

/* device status word bits */
#define DPFT_STATUS_NONFINITE 0x1u /* a JtJ / JtR reduction was not finite         */

/* return codes */
#define DPFT_OK            0
#define DPFT_E_INVALID    -1 /* bad descriptor / null pointer / unsupported shape */
#define DPFT_E_WORKSPACE  -2 /* workspace too small                                */
#define DPFT_E_HIP        -3 /* a HIP runtime call failed                          */

typedef struct DpftLevelDesc {
    int32_t B;       /* pairs in the batch                                    */
    int32_t C;       /* feature channels                                      */
    int32_t Cs;      /* uncertainty channels: 1 (broadcast) or C              */
    int32_t H, W;    /* level resolution                                      */
    int32_t iters;   /* Gauss-Newton iterations (reference: max_iter_per_pyr)  */
    uint32_t flags;  /* DPFT_REMOVE_TRU_SIGMA | DPFT_COMBINE_ICP | ...        */
    float icp_weight;/* ScaleNet('None') weight, 0.01 (algorithms.py:1563)    */
} DpftLevelDesc;

/* All tensors fp32 contiguous NCHW unless stated; nullable ones may be NULL. */
typedef struct DpftLevelTensors {
    const float* f0;      /* [B,C,H,W]  reference features                     */
    const float* f1;      /* [B,C,H,W]  target features                        */
    const float* s0;      /* [B,Cs,H,W] reference uncertainty                   */
    const float* s1;      /* [B,Cs,H,W] target uncertainty                      */
    const float* invD0;   /* [B,1,H,W]  reference inverse depth                 */
    const float* invD1;   /* [B,1,H,W]  target inverse depth                    */
    const float* depth0;  /* [B,1,H,W]  raw depth (COMBINE_ICP only)            */
    const float* depth1;  /* [B,1,H,W]  raw depth (COMBINE_ICP only)            */
    const uint8_t* mask0; /* [B,1,H,W]  object mask of frame 0, nullable        */
    const uint8_t* mask1; /* [B,1,H,W]  object mask of frame 1, nullable        */
    const float* K;       /* [B,4]      (fx,fy,cx,cy) of THIS level             */
    uint32_t* status;     /* [1]        device status word, OR-ed, never cleared */
    const float* weights; /* [B,1,H,W]  per-pixel M-estimator weights, nullable;
                             DPFT_NO_UNCERTAINTY only (TrustRegionBase with a learned
                             DeepRobustEstimator, algorithms.py:71-76, 1631-1632)  */
} DpftLevelTensors;

/* Bytes of workspace the level needs (>= 256-byte aligned pointer expected).
 * The workspace must be ZERO-FILLED before its first use (hipMemsetAsync):
 * it holds the completion counters of the in-kernel finalize, which every call
 * leaves at zero again.  One workspace serves one stream at a time. */
size_t dpft_workspace_size(const DpftLevelDesc* desc);

/*
 * Run desc->iters Gauss-Newton iterations at one pyramid level.
 * R [B,3,3] (row-major) and t [B,3] are read and updated in place (fp32).
 * jtj_out [B,36] / jtr_out [B,6] (nullable) receive the LAST iteration's
 * undamped JtJ / JtR (the reference's `inv_sigma_ksi`, algorithms.py:716-721).
 * NCHW features (no DPFT_FEATURES_C4) with C % 16 == 0, one sigma plane (or
 * DPFT_NO_UNCERTAINTY) and iters >= 2 are packed once on entry into the workspace
 * (dpft_workspace_size counts the two copies) and solved by the channel-quad kernels:
 * the same poses, bit for bit, as a call handed the packed features.
 */
int dpft_ic_solve_level(const DpftLevelDesc* desc, const DpftLevelTensors* tensors,
                        float* R, float* t, float* jtj_out, float* jtr_out,
                        void* workspace, size_t workspace_bytes, void* hip_stream);

/*
 * A whole coarse-to-fine solve: descs[0] / tensors[0] is the COARSEST level, the last
 * one level 0 (LeastSquareTracking.forward runs tr_update3 .. tr_update0,
 * LeastSquareTracking.py:349-445), each desc->iters iterations, R / t chained in place.
 * All levels share B, C, Cs, iters and flags (their K already divided by 2^level) and
 * one workspace of the largest level's size.  With DPFT_REMOVE_TRU_SIGMA every desc
 * carries DPFT_EXT_SLOT (<= 4 levels): the sigma0 extrema of all levels come from one
 * pre-pass (dpft_sigma_extrema_levels), then each level runs as dpft_ic_solve_level.
 */
int dpft_ic_solve_pyramid(const DpftLevelDesc* descs, const DpftLevelTensors* tensors, int32_t levels,
                          float* R, float* t, void* workspace, size_t workspace_bytes, void* hip_stream);

/*
 * One iteration (residual -> Jacobian -> JtJ/JtR -> damped solve -> update).
 * `first`: bit 0 (DPFT_ITER_FIRST) must be set on the first iteration of a level
 * (it computes the per-level sigma0 extrema); bit 2 (DPFT_ITER_NO_UPDATE) only writes
 * jtj_out / jtr_out (the damped solve and the pose update are skipped); bit 1
 * (DPFT_ITER_REVERSE) walks the
 * level in the reverse order (dpft_ic_solve_level sets it on odd iterations, so
 * an iteration starts on the bytes the previous one read last, still in the
 * Infinity Cache; same arithmetic, different fp32 summation grouping).
 * invalid_out [B] (nullable, int32) receives the number of invalid pixels of
 * this iteration's residual.
 */
#define DPFT_ITER_FIRST 1u
#define DPFT_ITER_REVERSE 2u
#define DPFT_ITER_NO_UPDATE 4u /* normal equations only (jtj_out / jtr_out), R / t untouched:
                                  the residual-volume samples of DirectSolverNet 'Direct-ResVol'
                                  (algorithms.py:1668-1685)                                    */
int dpft_ic_iterate(const DpftLevelDesc* desc, const DpftLevelTensors* tensors,
                    float* R, float* t, float* jtj_out, float* jtr_out, int32_t* invalid_out,
                    int first, void* workspace, size_t workspace_bytes, void* hip_stream);

/*
 * Residual-only evaluation at a fixed pose (forward_residuals):
 * loss[b] = sum_valid sum_c w_res^2 [+ (w_icp r_icp)^2] / (H*W - #invalid).
 */
int dpft_ic_residual_level(const DpftLevelDesc* desc, const DpftLevelTensors* tensors,
                           const float* R, const float* t, float* loss,
                           void* workspace, size_t workspace_bytes, void* hip_stream);

/*
 * Residual-only evaluation of n_poses poses per pair in one launch (the
 * convergence-basin sweep, convergence_basin.py:85-475, with the feature
 * pyramid computed once instead of once per pose as LeastSquareTracking.py:620
 * does).  R [n_poses,B,3,3], t [n_poses,B,3], loss [n_poses,B]; pose p is
 * evaluated as one reference call over the batch (its own batch-global
 * truncated-sigma extrema).  Workspace: dpft_residual_poses_workspace_size.
 */
size_t dpft_residual_poses_workspace_size(const DpftLevelDesc* desc, int32_t n_poses);
int dpft_ic_residual_poses(const DpftLevelDesc* desc, const DpftLevelTensors* tensors, int32_t n_poses,
                           const float* R, const float* t, float* loss,
                           void* workspace, size_t workspace_bytes, void* hip_stream);

/*
 * The batch-global sigma0 min / max of every level of a pyramid (the truncated-sigma
 * masks' pose-independent half, algorithms.py:1976-1977) in ONE launch, into the
 * workspace slots named by each descriptor's DPFT_EXT_SLOT.  The levels then run with
 * DPFT_EXTREMA_READY.  Replaces one min/max launch per level (LeastSquareTracking.py:
 * 349-445 solves 4 levels per pair).  All levels must share `workspace`.
 */
int dpft_sigma_extrema_levels(const DpftLevelDesc* descs, const DpftLevelTensors* tensors, int32_t levels,
                              void* workspace, size_t workspace_bytes, void* hip_stream);

/*
 * The IC tracker's residual map at pose (R, t) (compute_warped_residual,
 * algorithms.py:1919-1957; DPFT_NO_UNCERTAINTY): out [B,C,H,W] fp32 NCHW =
 * bilinear(f1, warp) - f0 with 1e-3 on occluded / masked pixels, occ_out [B,1,H,W]
 * uint8 (nullable) = those pixels.  The input of the learned M-estimator
 * (DeepRobustEstimator 'MultiScale2w', algorithms.py:1467-1477) and of its weighted
 * residual loss (forward_residuals 125-139).
 */
int dpft_ic_residual_map(const DpftLevelDesc* desc, const DpftLevelTensors* tensors, const float* R, const float* t,
                         float* out, uint8_t* occ_out, void* workspace, size_t workspace_bytes, void* hip_stream);

/* Kernel-only timing hook for the roofline: launch ONLY the fused residual +
 * Jacobian + normal-equation kernel (no finalize), using the sigma0 extrema a
 * previous dpft_ic_iterate(first=1) left in the workspace.  Used by tools/kbench.py.
 * With DPFT_COMBINE_ICP on the channel-quad path (DPFT_FEATURES_C4, C % 16 == 0) this is
 * TWO launches -- the point-to-plane pass (icp_records_kernel) and the U_IC reduce -- and
 * the per-workgroup records it leaves hold the U_IC terms only: the ICP records are merged
 * by the finalize (pair_reduce2), which this hook does not run.  Timing only: its records
 * are not the level's normal equations on that path. */
int dpft_ic_reduce_only(const DpftLevelDesc* desc, const DpftLevelTensors* tensors,
                        const float* R, const float* t,
                        void* workspace, size_t workspace_bytes, void* hip_stream);

/* Debug / test hook: per-pixel dump out[B,5,H,W] = (u, v, sigma_r ch0, sigma0 ch0,
 * occlusion|mask invalid) at the given pose.  Not on the solve path. */
int dpft_ic_debug_pixels(const DpftLevelDesc* desc, const DpftLevelTensors* tensors,
                         const float* R, const float* t, float* out,
                         void* workspace, size_t workspace_bytes, void* hip_stream);

/*
 * Depth preprocessing of LeastSquareTracking._preprocess (LeastSquareTracking.py:
 * 653-661, 669-676): invD = clamp(1/depth, 0, 10) with the batch-global min and
 * then max zeroed, and the max-pool pyramids (algorithms.py:1201-1219) of invD
 * and (depth_out non-NULL, for ICP) of the raw depth.  depth [B,1,H,W];
 * invd_out / depth_out: host arrays of `levels` device pointers, level l is
 * [B,1,H>>l,W>>l].  Workspace: dpft_preprocess_workspace_size() bytes, zero-filled
 * once (shared with the solver's workspace is fine on the same stream).
 */
size_t dpft_preprocess_workspace_size(void);
int dpft_preprocess_depth(const float* depth, int32_t B, int32_t H, int32_t W, int32_t levels,
                          float* const* invd_out, float* const* depth_out,
                          void* workspace, size_t workspace_bytes, void* hip_stream);

/*
 * Feature relayout for DPFT_FEATURES_C4: src [B,C,H,W] (NCHW, the encoder's
 * output, LeastSquareTracking.py:679-680) -> dst [B,C/4,H,W,4], C % 4 == 0.
 * Pose-independent: done once per level per forward, every Gauss-Newton iteration
 * and every residual pose of the level reads the packed copy.  src != dst.
 */
int dpft_pack_features(const float* src, float* dst, int32_t B, int32_t C, int32_t H, int32_t W, void* hip_stream);

/*
 * The same relayout from a channels_last map: src [B,H,W,C] (NHWC; the encoder run in
 * channels_last memory format, `torch.channels_last`) -> dst [B,C/4,H,W,4].  One pass,
 * instead of a transposition to NCHW followed by dpft_pack_features.  16-byte aligned.
 */
int dpft_pack_features_nhwc(const float* src, float* dst, int32_t B, int32_t C, int32_t H, int32_t W,
                            void* hip_stream);

/*
 * Encoder block epilogue in eval mode (reference submodules.py:25-39, convLayer:
 * conv -> BatchNorm2d(running statistics) -> ELU), in place on the conv output x of n
 * floats: x = elu(x * a[c] + b[c]) with a = weight / sqrt(running_var + eps),
 * b = bias - running_mean * a (chan = [a | b], 2C floats, device).  nhwc = 1: x is
 * channels_last (channel = index % C; C % 4 == 0, inner = 1); nhwc = 0: NCHW with inner =
 * H*W (channel = index / inner % C; inner % 4 == 0).  x 16-byte aligned.
 */
int dpft_bn_elu(float* x, const float* chan, int64_t n, int32_t C, int64_t inner, int32_t nhwc, void* hip_stream);

/*
 * The feature heads' epilogue writing the solver's layout: the eval-mode BatchNorm + ELU
 * of dpft_bn_elu applied to a channels_last conv output x [B,H,W,C] (the f_conv heads,
 * reference algorithms.py:1273-1277 with convLayer submodules.py:25-39), written OUT OF
 * PLACE to the channel-quad layout out [B,C/4,H,W,4] (DPFT_FEATURES_C4) -- the same values
 * dpft_bn_elu followed by dpft_pack_features_nhwc give, in one read and one write instead of
 * two of each.  C % 4 == 0; x, out 16-byte aligned, not aliased.
 */
int dpft_bn_elu_pack(const float* x, const float* chan, float* out, int32_t B, int32_t C, int32_t H, int32_t W,
                     void* hip_stream);

/*
 * Jacobian API, materialised -- the reference solver's methods that the fused solve
 * never needs (it keeps J in registers); kept for callers and tests that inspect J.
 *  dpft_feature_gradient    feature_gradient (algorithms.py:1844-1865): unit-normalised
 *                           replicate-padded Sobel, f [B,C,H,W] -> grad [B,C,2,H,W].
 *  dpft_warp_jacobian       compute_jacobian_warping (1884-1917) at the origin:
 *                           invD0, px, py [B,1,H,W], K [B,4] -> Jx, Jy [B,HW,6].
 *  dpft_inverse_jacobian    compose_inverse_jacobians (867-887) + compute_jacobian_dIdp
 *                           (1867-1882): res, sigma [B,C,H,W], sigma0 [B,Cs,H,W],
 *                           grad_f0 [B,C,2,H,W], grad_sigma0 [B,Cs,2,H,W] (Cs = 1 or C)
 *                           -> J [B,C,HW,6] (not masked, as the reference).
 *  dpft_normal_equations    compute_jtj / compute_jtr (812-834): J [B,n,6], r [B,n]
 *                           (NULL: JtJ only) -> jtj [B,6,6], jtr [B,6]; fp64 partials in
 *                           a fixed order (deterministic); workspace of
 *                           dpft_normal_equations_workspace_size(B) bytes.
 */
int dpft_feature_gradient(const float* f, float* grad, int32_t B, int32_t C, int32_t H, int32_t W,
                          void* hip_stream);
int dpft_warp_jacobian(const float* invD0, const float* K, const float* px, const float* py, float* Jx, float* Jy,
                       int32_t B, int32_t H, int32_t W, void* hip_stream);
int dpft_inverse_jacobian(const float* res, const float* sigma, const float* sigma0, const float* grad_f0,
                          const float* grad_sigma0, const float* Jx, const float* Jy, float* J, int32_t B, int32_t C,
                          int32_t Cs, int32_t H, int32_t W, void* hip_stream);
size_t dpft_normal_equations_workspace_size(int32_t B);
int dpft_normal_equations(const float* J, const float* r, int64_t n, int32_t B, float* jtj, float* jtr, void* ws,
                          size_t ws_bytes, void* hip_stream);

/*
 * Damped inverse-compositional update of 'Direct-ResVol' (DirectSolverNet,
 * algorithms.py:1644-1691, then inverse_update_pose 2017-2054), for S damping choices
 * per pair at once: H[s,b] = JtJ[b] + diag(diag_add[s,b]) + 1e-6 tr(JtJ[b]) I,
 * xi = H^-1 JtR[b] (fp64 Cholesky), R_out[s,b] = R[b] Exp(-w), t_out[s,b] =
 * R[b] (-Exp(-w) v) + t[b].  jtj [B,6,6], jtr [B,6], diag_add [S,B,6] (NULL: none),
 * R [B,3,3], t [B,3] -> R_out [S,B,3,3], t_out [S,B,3]; outputs must not alias inputs.
 * The residual-volume trial poses use diag_add = lambda_s diag(JtJ), the final step the
 * MLP's damping.
 */
int dpft_ic_damped_update(const float* jtj, const float* jtr, const float* diag_add, int32_t S, int32_t B,
                          const float* R, const float* t, float* R_out, float* t_out, void* hip_stream);

/*
 * Diagnostic, not on the solve path: read `bytes` (16-byte aligned) of device memory
 * once with 16-byte loads (non-temporal if `nontemporal`), four in flight per lane,
 * 4096 workgroups; writes dpft_read_probe_out_floats() partial sums to `out`.  Timed by
 * bench.py as the measured HBM read ceiling the level-0 roofline is reported against
 * beside the 8 TB/s spec.
 */
size_t dpft_read_probe_out_floats(void);
int dpft_read_probe(const void* buf, size_t bytes, int32_t nontemporal, float* out, void* hip_stream);
/* Diagnostic: copy `bytes` (16-byte aligned src / dst) with 16-byte loads and stores -- mode 0:
 * one float4 per thread (MI355X_MICROARCH.md's float4 copy), mode 1: grid-stride, non-temporal,
 * four in flight per lane; bench.py reports the faster (read + write) rate as the measured copy
 * ceiling. */
int dpft_copy_probe(const void* src, void* dst, size_t bytes, int32_t mode, void* hip_stream);

int dpft_version(void);            /* DPFT_ABI_VERSION */
const char* dpft_last_error(void); /* thread-local message of the last failure */

#ifdef __cplusplus
}
#endif
#endif /* DPFT_IC_H */
