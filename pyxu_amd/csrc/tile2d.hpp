// Shared machinery of the LDS-tiled 2-D separable-stencil kernels (pgd_tv2d.hip, pds3d.hip):
// tile geometry, LDS layout, register-blocked Toeplitz sweeps and the exact zero-boundary
// corrections of G = H^T H (see the derivation at the top of pgd_tv2d.hip).
#pragma once
#include "common.hpp"

namespace pxa {
namespace tile2d {

constexpr int TY = 32;
constexpr int TX = 64;
constexpr int kThreads = 256;
constexpr int kMaxR = 8;
constexpr int kMaxG = 4 * kMaxR + 1;
constexpr int kKT = 2 * kMaxR + 2;  // per-axis stride of the LDS tap copy (edge tiles)

__host__ __device__ constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ constexpr int rup(int a, int b) { return cdiv(a, b) * b; }

template <typename T, int R>
struct Layout {
  static constexpr int V = kVecN<T>;  // elements per 16-B vector (4 fp32, 2 fp64)
  static constexpr bool F32 = sizeof(T) == 4;
  static constexpr int CA = rup(2 * R, V);  // A column halo (vector aligned)
  static constexpr int AR = TY + 4 * R;     // A rows
  static constexpr int AC = TX + 2 * CA;    // A columns = PT rows
  static constexpr int NGA = AC / V;        // phase 0: AR x NGA vectors
  static constexpr int NA = TY / V;         // row groups (pass A and pass B)
  static constexpr int NB = AC / V;         // pass A column groups
  static constexpr int CW = F32 ? 2 : 1;    // pass B: output columns per item
  static constexpr int NCB = TX / CW;       // pass B column items
  static constexpr int pad_to(int w, int m, int res) {
    int p = w;
    while (F32 && (p % m) != res) p += V;
    return p;
  }
  static constexpr int AP = pad_to(AC, 32, 28);   // A pitch (elements)
  static constexpr int PTP = F32 ? TY + 8 : TY;  // PT pitch (elements): conflict-free with pass_b_item
  // pass B item of linear index `it`: row group a, column item cb.  fp32: each 32-lane half of a wave
  // takes 4 row groups x 8 column items, so that both the G1 sweep (ds_read_b128 of PT) and the yk
  // window reads of the TV stencil (ds_read_b64 of A, row groups 4 apart collide mod 64 banks) are
  // conflict-free under the MI355X_MICROARCH.md bank model (scripts/ldsbank.py)
  __device__ static inline void pass_b_item(int it, int& a, int& cb) {
    if constexpr (F32 && NA == 8) {
      a = (it & 3) + 4 * ((it >> 5) & 1);
      cb = ((it >> 2) & 7) + 8 * (it >> 6);
    } else {
      a = it % NA;
      cb = it / NA;
    }
  }
  static constexpr int N0 = AR * NGA, NPA = NA * NB, NPB = NA * NCB;
  static constexpr size_t BYTES = (size_t)(AR * AP + AC * PTP + 2 * kKT) * sizeof(T);
};

template <typename T, int V>
__device__ inline void ld_vec(const T* p, T (&v)[V]) {
  using VT = typename Vec4<T>::type;
  *reinterpret_cast<VT*>(v) = *reinterpret_cast<const VT*>(p);
}
template <typename T, int V>
__device__ inline void st_vec(T* p, const T (&v)[V]) {
  using VT = typename Vec4<T>::type;
  *reinterpret_cast<VT*>(p) = *reinterpret_cast<const VT*>(v);
}

template <typename T>
__device__ inline T apply_prox(int prox, T z, T pw) {
  if (prox == 1) return fmax(z, T(0));  // PositiveOrthant: clip(0, None)
  if (prox == 2) {                       // L1: sign(z) * max(|z| - pw, 0)
    T m = (z < T(0) ? -z : z) - pw;
    m = m > T(0) ? m : T(0);
    return z < T(0) ? -m : m;
  }
  return z;
}

// Packed-arithmetic unit: fp32 pairs (v_pk_fma_f32), fp64 scalars.
template <typename T>
struct Pk {
  using type = T;
  static constexpr int W = 1;
  __device__ static type splat(T v) { return v; }
};
template <>
struct Pk<float> {
  typedef float type __attribute__((ext_vector_type(2)));
  static constexpr int W = 2;
  __device__ static type splat(float v) { return type{v, v}; }
};

// Register-blocked sweep along the leading axis of a [m][pitch PS] source: for NO outputs along the
// sweep and one V-vector across it, out[o][v] = sum_{t=0}^{4R} g[t] src[(o + t) * PS + v].
// D = 0: the compiler schedules the NO + 4R row loads (it hoists most of them: ~4 VGPRs per row live at once).
// D > 0: at most D rows in flight -- row j + D is loaded when row j is consumed, and a scheduling barrier (only
// VALU / SALU may cross it) keeps the LDS reads in that order -- so a sweep holds ~4 (D + 1) row registers: the
// PGD strip kernel's budget for its prefetched window rows.  Same FMAs in the same order: same bits.
template <typename T, int R, int NO, int PS, int D = 0>
__device__ inline void sweep(const T* __restrict__ src, const T* __restrict__ g, T (&out)[NO][kVecN<T>]) {
  constexpr int V = kVecN<T>;
  using P = typename Pk<T>::type;
  constexpr int NP = V / Pk<T>::W;
  using VT = typename Vec4<T>::type;
  constexpr int NJ = NO + 4 * R;
  P acc[NO][NP];
#pragma unroll
  for (int o = 0; o < NO; ++o)
#pragma unroll
    for (int h = 0; h < NP; ++h) acc[o][h] = Pk<T>::splat(T(0));
  if constexpr (D > 0) {
    VT ring[D];
#pragma unroll
    for (int j = 0; j < D && j < NJ; ++j) ring[j] = *reinterpret_cast<const VT*>(src + j * PS);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const VT t = ring[j % D];
      if (j + D < NJ) ring[j % D] = *reinterpret_cast<const VT*>(src + (j + D) * PS);
      P row[NP];
      __builtin_memcpy(&row[0], &t, sizeof(VT));
#pragma unroll
      for (int o = 0; o < NO; ++o) {
        const int k = j - o;
        if (k >= 0 && k <= 4 * R) {
          const P gg = Pk<T>::splat(g[k]);
#pragma unroll
          for (int h = 0; h < NP; ++h) acc[o][h] = gg * row[h] + acc[o][h];
        }
      }
      __builtin_amdgcn_sched_barrier(0x6);  // VALU and SALU may move across, LDS reads may not
    }
#pragma unroll
    for (int o = 0; o < NO; ++o) __builtin_memcpy(&out[o][0], &acc[o][0], sizeof(T) * V);
    return;
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const VT t = *reinterpret_cast<const VT*>(src + j * PS);
    P row[NP];
    __builtin_memcpy(&row[0], &t, sizeof(VT));
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      const int k = j - o;
      if (k >= 0 && k <= 4 * R) {
        const P gg = Pk<T>::splat(g[k]);
#pragma unroll
        for (int h = 0; h < NP; ++h) acc[o][h] = gg * row[h] + acc[o][h];
      }
    }
  }
#pragma unroll
  for (int o = 0; o < NO; ++o) __builtin_memcpy(&out[o][0], &acc[o][0], sizeof(T) * V);
}

// Boundary rows of G along one axis, as a correction of the Toeplitz sweep.  The sweep evaluates
// sum_p k[i-p] (H y)[p] over ALL p, i.e. including the R "ghost" positions p outside [0, n) where the
// zero-padded H y is still non-zero; the exact G = H^T H only sums p inside [0, n), so
//   (G y)[i] = sweep[i] - sum_{ghost p, |i - p| <= R} k[i - p] (H y)[p].
// acc[o][v]: NO outputs along the sweep axis at positions i0 + o, one V-vector across it;
// the V-vector of position q along the sweep axis is at src + (q - q0) * PS (zero outside [0, n));
// k: the taps (compile-time indices), kt: the same taps in LDS (runtime indices).
template <typename T, int R, int NO, int PS>
__device__ inline void ghost_fix(int i0, int n, int q0, const T* __restrict__ src, const T* __restrict__ k,
                                 const T* __restrict__ kt, T (&acc)[NO][kVecN<T>]) {
  constexpr int V = kVecN<T>;
  using VT = typename Vec4<T>::type;
#pragma unroll
  for (int side = 0; side < 2; ++side) {
    const int pg = side == 0 ? -R : n;  // first ghost position on this side
    const bool hit = side == 0 ? (i0 < R) : (i0 + NO - 1 >= n - R && i0 < n);
    if (!hit) continue;
    T gh[R][V];  // (H y)[pg + m] across the vector
#pragma unroll
    for (int m = 0; m < R; ++m) {
      const int pp = pg + m;
#pragma unroll
      for (int v = 0; v < V; ++v) gh[m][v] = T(0);
      if (pp >= i0 - R && pp <= i0 + NO - 1 + R) {  // used by some output (keeps reads inside the window)
#pragma unroll
        for (int s = -R; s <= R; ++s) {
          T w[V];
          const VT t = *reinterpret_cast<const VT*>(src + (pp + s - q0) * PS);
          __builtin_memcpy(&w[0], &t, sizeof(VT));
#pragma unroll
          for (int v = 0; v < V; ++v) gh[m][v] = fma(k[s + R], w[v], gh[m][v]);
        }
      }
    }
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      const int i = i0 + o;
      if (i >= n || (side == 0 ? i >= R : i < n - R)) continue;
#pragma unroll
      for (int m = 0; m < R; ++m) {
        const int t = i - (pg + m);
        if (t < -R || t > R) continue;
        const T kk = kt[t + R];
#pragma unroll
        for (int v = 0; v < V; ++v) acc[o][v] = fma(-kk, gh[m][v], acc[o][v]);
      }
    }
  }
}

// Boundary columns of the in-plane pass B (edge-column tiles), computed cooperatively into LDS:
// GH[side][m][r] = sum_s k[s] PT[ghost column pg + m + s][tile row r] for the R zero-padded ghost
// columns pg + m on each side (pg = -R, n) -- ghost_fix()'s gh with the same fma order.  With ghost_fix()
// the few lanes owning columns within R of the border compute them all, one 2R+1-tap sum per ghost
// column and lane: one wave then runs thousands of cycles past the others (measured by the PGD
// kernels' s_memtime trace).  Followed by a barrier, then ghost_fix_pre() in pass B.
template <typename T, int R>
__device__ inline void ghost_cols_coop(const T* __restrict__ k, const T* PT, T* GH, int tx0, int n, int lt = threadIdx.x,
                                       int nthr = kThreads) {
  using L = Layout<T, R>;
  for (int t = lt; t < 2 * R * TY; t += nthr) {
    const int side = t / (R * TY), m = (t / TY) % R, r = t % TY;
    const int row = (side == 0 ? -R : n) + m - (tx0 - L::CA);  // PT row of the ghost column
    T g = T(0);
    if (row - R >= 0 && row + R < L::AC) {  // else no output of this tile uses it
#pragma unroll
      for (int q = -R; q <= R; ++q) g = fma(k[q + R], PT[(row + q) * L::PTP + r], g);
    }
    GH[(side * R + m) * TY + r] = g;
  }
}

// ghost_fix()'s correction step with precomputed ghost terms: outputs i0 .. i0 + NO - 1 along the sweep
// axis (n positions), one V-vector across it from position cc of the GH rows (pitch GP)
template <typename T, int R, int NO, int GP>
__device__ inline void ghost_fix_pre(int i0, int n, int cc, const T* __restrict__ GH, const T* __restrict__ kt,
                                     T (&acc)[NO][kVecN<T>]) {
  constexpr int V = kVecN<T>;
#pragma unroll
  for (int side = 0; side < 2; ++side) {
    const int pg = side == 0 ? -R : n;
    const bool hit = side == 0 ? (i0 < R) : (i0 + NO - 1 >= n - R && i0 < n);
    if (!hit) continue;
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      const int i = i0 + o;
      if (i >= n || (side == 0 ? i >= R : i < n - R)) continue;
#pragma unroll
      for (int m = 0; m < R; ++m) {
        const int t = i - (pg + m);
        if (t < -R || t > R) continue;
        const T kk = kt[t + R];
        T gh[V];
        const auto* src = GH + (side * R + m) * GP + cc;
#pragma unroll
        for (int v = 0; v < V; ++v) gh[v] = src[v];
#pragma unroll
        for (int v = 0; v < V; ++v) acc[o][v] = fma(-kk, gh[v], acc[o][v]);
      }
    }
  }
}

// byte offset / size of the ghost-term region the tile kernels append to the Layout carve
template <typename T, int R>
constexpr size_t kGhOff = (Layout<T, R>::BYTES + 15) / 16 * 16;
template <typename T, int R>
constexpr size_t kGhBytes = (size_t)2 * R * TY * sizeof(T);

// Global V-vector load at an element offset whose alignment is known at compile time.
template <typename T>
__device__ inline void ld_pair(const T* __restrict__ p, T (&v)[2]) {
  if constexpr (sizeof(T) == 4) {
    const float2 t = *reinterpret_cast<const float2*>(p);
    v[0] = t.x;
    v[1] = t.y;
  } else {
    v[0] = p[0];
    v[1] = p[1];
  }
}

// Staged epilogue geometry: pass B parks its results in O (the PT region, free once all G sweeps are
// done), then the workgroup finishes the tile in row-major order, each 16-B vector of a tile row one
// lane (16 lanes per fp32 row): the global loads / stores of the epilogue are full 128-B lines instead
// of the pass-B item order's 64-B row pieces (measured on MI355X: a 2048^2 fp32 store in the item order
// 7.2 us, row-major 5.2 us).
template <typename T, int R>
struct Stage {
  using L = Layout<T, R>;
  static constexpr int V = L::V;
  static constexpr bool F32 = sizeof(T) == 4;
  // fp32: 64-dword rows with the 16-B chunks of row r XOR-swizzled by 2 (r / 4): the pass-B item-order
  // ds_write_b64 (rows 4a + u, column pairs of cb) hit 32 distinct banks per 16-lane group, and a
  // row-major ds_read_b128 group reads one whole row (64 contiguous dwords, permuted): both
  // conflict-free under the MI355X_MICROARCH.md §LDS bank model (scripts/ldsbank.py)
  static constexpr int OP = F32 ? TX : TX + 2;
  static constexpr int LPR = TX / V;          // lanes per tile row
  static constexpr int RPS = kThreads / LPR;  // rows per sweep
  static_assert(TY * OP <= L::AC * L::PTP, "O must fit in the PT region");
  __device__ static inline int idx(int r, int c) {
    if constexpr (F32) return r * OP + 4 * (((c >> 2) ^ (2 * (r >> 2))) & 15) + (c & 3);
    else return r * OP + c;
  }
  // row-major epilogue lane -> (tile row r0 of the first sweep, 16-B column vector cq).  fp32: each
  // ds_read_b128 lane group ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32) takes one row, so the reads
  // of O and of the yk window A are contiguous 64-dword runs whatever the pitch; global accesses of a
  // wave still cover 4 whole 256-B tile rows
  __device__ static inline void lane(int tid, int& r0, int& cq) {
    if constexpr (F32) {
      static_assert(TX == 64 && kThreads % 64 == 0, "fp32 lane map assumes 64-column tiles");
      const int ln = tid & 63, w = tid >> 6, h = ln >> 5, l = ln & 31;
      int g, pos;
      if (l < 4) g = 0, pos = l;
      else if (l < 12) g = 1, pos = l - 4;
      else if (l < 16) g = 0, pos = l - 8;
      else if (l < 20) g = 1, pos = l - 8;
      else if (l < 28) g = 0, pos = l - 12;
      else g = 1, pos = l - 16;
      r0 = 4 * w + 2 * h + g;
      cq = pos;
    } else {
      cq = tid % LPR;
      r0 = tid / LPR;
    }
  }
};

// XCD-aware tile order (speed only): XCD group g = blockIdx % 8 owns a contiguous band of tiles.
__device__ inline unsigned xcd_tile(unsigned bid, unsigned nb) {
  const unsigned q8 = nb >> 3, r8 = nb & 7u, g8 = bid & 7u;
  return g8 * q8 + (g8 < r8 ? g8 : r8) + (bid >> 3);
}

}  // namespace tile2d
}  // namespace pxa
