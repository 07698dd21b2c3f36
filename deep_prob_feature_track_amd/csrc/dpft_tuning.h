// dpft_tuning.h -- the numeric operating point of libdpft_ic.so's schedules (no code paths).
// The shipped build uses these defaults; tools/build_variants.py may override them with -D
// for A/B builds of the SAME kernels (DESIGN.md §4 records the sweeps behind each value).
#ifndef DPFT_TUNING_H
#define DPFT_TUNING_H

// channel-quad levels up to this many pixels per pair -> ic_split_kernel (levels 2, 3 at cfg2)
#ifndef DPFT_SPLIT_MAX_PIXELS
#define DPFT_SPLIT_MAX_PIXELS 40000
#endif
// ... and up to this many pixels per launch (all pairs of a grouped call)
#ifndef DPFT_SPLIT_MAX_LAUNCH_PIXELS
#define DPFT_SPLIT_MAX_LAUNCH_PIXELS 320000
#endif
// marching bands: weights 64 + skew / 64 - skew for the first / second dispatched half of a
// pair's waves (swept 0..22 in rounds 1-2: 10 fastest; round 3 with the cross-row f0
// prefetch, 64 pairs per launch: 0..3 fastest, within 0.5 % of each other, 10 -1.3 %)
#ifndef DPFT_MARCH_SKEW
#define DPFT_MARCH_SKEW 2
#endif
// marching band grid: idle waves allowed, in 64ths of a pair's waves (more idle waves than
// this and the hybrid or grid + pool split is used instead)
#ifndef DPFT_GRID_WASTE
#define DPFT_GRID_WASTE 4
#endif
// marching bands: at least this many rows per wave (0: no minimum) -- fewer workgroups per
// pair on short levels, whose bands otherwise spend two window rows of priming per band
#ifndef DPFT_MARCH_MIN_ROWS
#define DPFT_MARCH_MIN_ROWS 0
#endif
// marching quad loop: quads in flight (swept 2 / 3 / 4 / 6)
#ifndef DPFT_RING_Q
#define DPFT_RING_Q 4
#endif
// combine_ICP pass (icp_records_kernel): at most this many workgroups per reduce workgroup slot
#ifndef DPFT_ICP_SUB
#define DPFT_ICP_SUB 4
#endif
// sigma0 / depth extrema pass: workgroups and 16-byte loads in flight per thread
#ifndef DPFT_MM_GRID
#define DPFT_MM_GRID 128
#endif
#ifndef DPFT_MM_LOADS
#define DPFT_MM_LOADS 8
#endif
// diagnostic read / copy probes: workgroups (16 per CU) and 16-byte loads in flight per lane
#ifndef DPFT_PROBE_GRID
#define DPFT_PROBE_GRID 4096
#endif
#ifndef DPFT_PROBE_DEPTH
#define DPFT_PROBE_DEPTH 4
#endif

#endif  // DPFT_TUNING_H
