// pyxu_amd — shared helpers for the gfx950 kernels behind the C-ABI (include/pyxu_amd.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pyxu_amd.h"

namespace pxa {

constexpr int kWave = 64;  // CDNA wavefront width

// Launch geometry for streaming kernels: 256 threads, at most 8 blocks per CU (256 CUs).
constexpr int kBlock = 256;
constexpr int kMaxGrid = 256 * 8;

inline int grid_for(int64_t work_items, int per_block = kBlock) {
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > kMaxGrid) g = kMaxGrid;
  return (int)g;
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int last_launch_status() {
  hipError_t e = hipGetLastError();
  return (int)e;
}

template <typename T>
struct Vec4;
template <>
struct Vec4<float> {
  using type = float4;
};
template <>
struct Vec4<double> {
  using type = double2;  // 16 B per lane for both precisions
};

// Current value of a pxa_tuning() knob (abi.hip).
int tuning(int key);

// Workgroups of `kernel` resident on the current device at once (occupancy x CUs), rounded down to a multiple
// of 8 so that workgroup w of a persistent grid stays on XCD w % 8 for every unit it takes (>= 8).  Cached per
// (kernel, device, threads, LDS).
int resident_grid(const void* kernel, int threads, size_t lds);

// Elements per 16-byte vector.
template <typename T>
constexpr int kVecN = 16 / sizeof(T);

// DPP operand of one double (two 32-bit halves through the same lane permutation)
template <int CTRL>
__device__ inline double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// Sum of a double over the 64 lanes of a wave, the same value in every lane, in a fixed order: within each
// 16-lane row by DPP (quad butterfly, then row rotations by 4 and 8), then the four row sums read from
// lanes 0, 16, 32, 48 and added in ascending order.  No LDS round trips (a __shfl_down ladder is six
// ds_bpermute pairs in series).
__device__ inline double wave_sum_f64(double d) {
  d += dpp_f64<0xB1>(d);   // quad_perm [1,0,3,2]
  d += dpp_f64<0x4E>(d);   // quad_perm [2,3,0,1]: every lane holds its quad's sum
  d += dpp_f64<0x124>(d);  // row_ror 4
  d += dpp_f64<0x128>(d);  // row_ror 8: lane 16 r holds row r's sum
  double r[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    r[q] = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(d), 16 * q),
                            __builtin_amdgcn_readlane(__double2loint(d), 16 * q));
  return ((r[0] + r[1]) + r[2]) + r[3];
}

// One RelError statistic of the fused PGD step's per-(tile, wavefront) partials, by a whole kBlock-thread
// workgroup: thread t sums pr[2 k] for k = t, t + kBlock, ... in order, the wavefront folds by a shuffle-down
// tree, then thread 0 adds the kBlock / 64 wave results in order (`red`: kBlock / 64 doubles of LDS).  The
// result is valid in thread 0.  Shared by pxa_tile_partials_fold (reduce.hip) and the tile kernel's own
// last-workgroup fold (pgd_tv2d.hip), so both give the same bits.
struct PlainLoad {
  __device__ double operator()(const double* a) const { return *a; }
};
// WIDE (the fold kernel; not the tile kernel's own tail, where the 64 extra VGPRs spill): up to kFoldBatch *
// kBlock partials (8 192: a 2048^2 image) every thread issues all its loads before the first add (one memory
// round trip instead of four batches of eight; the partials were written by every XCD, so they come from the
// Infinity Cache, not this XCD's L2), same sum order, same bits.
constexpr int kFoldBatch = 32;
template <bool WIDE = false, typename Load = PlainLoad>
__device__ inline double fold_tile_stat(const double* __restrict__ pr, int64_t per_row, double* red, Load ld = Load{}) {
  double acc = 0.0;
  if (WIDE && per_row <= (int64_t)kFoldBatch * kBlock) {
    double v[kFoldBatch];
#pragma unroll
    for (int j = 0; j < kFoldBatch; ++j) {
      const int64_t k = threadIdx.x + (int64_t)j * kBlock;
      v[j] = k < per_row ? ld(pr + 2 * k) : 0.0;
    }
#pragma unroll
    for (int j = 0; j < kFoldBatch; ++j)
      if (threadIdx.x + (int64_t)j * kBlock < per_row) acc += v[j];
  } else {
#pragma unroll 8
    for (int64_t k = threadIdx.x; k < per_row; k += kBlock) acc += ld(pr + 2 * k);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = acc;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < kBlock / kWave; ++i) t += red[i];
  __syncthreads();  // red may be reused by the next statistic
  return t;
}

// CG iteration tail partition (cg.hip): the <p, A p> and ||r'||^2 partials of a row come from cg_blocks(n)
// workgroups of kBlock threads, block b owning elements [b chunk, (b + 1) chunk), chunk = ceil(n / blocks),
// thread t summing elements lo + t, lo + t + kBlock, ... in order, then cg_block_sum.  Shared by cg.hip and
// the dense normal operator's fused reduction (dense.hip), so that both give the same bits.
constexpr int kCgBlocks = 64;
inline int cg_blocks(int64_t n) { return (int)(n < (int64_t)kCgBlocks * kBlock ? (n + kBlock - 1) / kBlock : kCgBlocks); }

// shuffle-down fold per wavefront, then thread 0 adds the kBlock / 64 wave results in order (valid in thread
// 0); every thread of the workgroup calls it, only the first kBlock threads' values count.
__device__ inline double cg_block_sum(double v, double* sh) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0 && w < kBlock / kWave) sh[w] = v;
  __syncthreads();
  double r = 0.0;
  if (threadIdx.x == 0) {
    r = sh[0];
    for (int k = 1; k < kBlock / kWave; ++k) r += sh[k];
  }
  return r;
}

}  // namespace pxa

// dtype dispatch: `code` is PXA_F32 / PXA_F64.
#define PXA_DISPATCH(code, T, ...)                 \
  do {                                             \
    if ((code) == PXA_F32) {                       \
      using T = float;                             \
      __VA_ARGS__;                                 \
    } else if ((code) == PXA_F64) {                \
      using T = double;                            \
      __VA_ARGS__;                                 \
    } else {                                       \
      return PXA_ERR_DTYPE;                        \
    }                                              \
  } while (0)

#define PXA_CHECK_ARG(cond)        \
  do {                             \
    if (!(cond)) return PXA_ERR_ARG; \
  } while (0)
