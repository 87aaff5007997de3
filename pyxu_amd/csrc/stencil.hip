// Stencil family: separable-axis passes, N-D stencils, Pad / Pad^T / Trim / Trim^T.
//
// Semantics follow the reference exactly (see include/pyxu_amd.h); the constant-mode path
// (zero_partial = 0) evaluates Trim o S o Pad without ever materialising the padded array.
// Memory-bound: one thread per output, lanes contiguous along the last (fastest) axis so every
// tap load is a coalesced row segment; tap re-reads are served by L1/L2.
#include "common.hpp"

namespace pxa {
namespace {

struct Geom {
  int nd;
  int64_t n[PXA_MAX_DIM];
  int64_t st[PXA_MAX_DIM];  // element strides (row-major)
  int64_t size;             // prod(n)
};

inline bool make_geom(int ndim, const int64_t* shape, Geom& g) {
  if (ndim < 1 || ndim > PXA_MAX_DIM || shape == nullptr) return false;
  g.nd = ndim;
  int64_t s = 1;
  for (int i = ndim - 1; i >= 0; --i) {
    if (shape[i] < 1) return false;
    g.n[i] = shape[i];
    g.st[i] = s;
    s *= shape[i];
  }
  for (int i = ndim; i < PXA_MAX_DIM; ++i) {
    g.n[i] = 1;
    g.st[i] = 0;
  }
  g.size = s;
  return true;
}

template <typename T>
struct AxisTaps {
  int n;
  int off[PXA_MAX_TAPS];
  T coef[PXA_MAX_TAPS];
};

// ------------------------------------------------------------------ one separable-axis pass
template <typename T, bool ZERO_PARTIAL>
__global__ void __launch_bounds__(kBlock) axis_kernel(int64_t stack, Geom g, int axis, AxisTaps<T> tp,
                                                      const T* __restrict__ x, int64_t xs, T* __restrict__ y,
                                                      int64_t ys, T beta) {
  const int64_t total = stack * g.size;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t sa = g.st[axis], na = g.n[axis];
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    int64_t s = t / g.size, r = t - s * g.size;
    int64_t ca = (r / sa) % na;
    const T* xr = x + s * xs + r;
    T acc = T(0);
    bool inside = true;
    for (int q = 0; q < tp.n; ++q) {
      int64_t c = ca + tp.off[q];
      if (c >= 0 && c < na) {
        acc = fma(tp.coef[q], xr[(int64_t)tp.off[q] * sa], acc);
      } else if (ZERO_PARTIAL) {
        inside = false;
      }
    }
    if (ZERO_PARTIAL && !inside) acc = T(0);
    T* yp = y + s * ys + r;
    *yp = (beta == T(0)) ? acc : acc + beta * (*yp);
  }
}

// Vector form of one separable-axis pass (round 4): a thread owns V consecutive elements of the last axis;
// the coordinate along the pass axis and the boundary tests are computed once per vector (the scalar
// kernel above spent ~10 VALU per tap and element on 64-bit index math: 0.088 ms for a 13-tap Gaussian on
// 2048^2, against ~8 us of HBM time); off-last-axis taps are whole-vector loads, last-axis taps read the
// vector's neighbours (L1).  Same sums in the same tap order, one fma each.
template <typename T, bool ZERO_PARTIAL, bool LAST>
__global__ void __launch_bounds__(kBlock) axis_vec_kernel(int64_t stack, Geom g, int axis, AxisTaps<T> tp,
                                                          const T* __restrict__ x, int64_t xs, T* __restrict__ y,
                                                          int64_t ys, T beta) {
  constexpr int V = kVecN<T>;
  using VT = typename Vec4<T>::type;
  const int64_t nvec = g.size / V, total = stack * nvec;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t sa = g.st[axis], na = g.n[axis];
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t s = t / nvec, r = (t - s * nvec) * V;
    const int64_t ca = (r / sa) % na;  // LAST: the first element's column
    const T* xr = x + s * xs + r;
    T acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = T(0);
    bool inside = true;
    for (int q = 0; q < tp.n; ++q) {
      const int o = tp.off[q];
      const T cq = tp.coef[q];
      if constexpr (!LAST) {
        const int64_t c = ca + o;
        if (c >= 0 && c < na) {
          T v[V];
          *reinterpret_cast<VT*>(v) = *reinterpret_cast<const VT*>(xr + (int64_t)o * sa);
#pragma unroll
          for (int e = 0; e < V; ++e) acc[e] = fma(cq, v[e], acc[e]);
        } else if (ZERO_PARTIAL) {
          inside = false;
        }
      } else {
        if (ca + o >= 0 && ca + o + V <= na) {  // the whole shifted vector inside the row
#pragma unroll
          for (int e = 0; e < V; ++e) acc[e] = fma(cq, xr[o + e], acc[e]);
        } else {
#pragma unroll
          for (int e = 0; e < V; ++e) {
            const int64_t c = ca + e + o;
            if (c >= 0 && c < na) acc[e] = fma(cq, xr[o + e], acc[e]);
          }
        }
      }
    }
    T out[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      T a = acc[e];
      if (ZERO_PARTIAL) {
        bool in = inside;
        if (LAST) {  // per element: every tap inside its row
          for (int q = 0; q < tp.n; ++q) {
            const int64_t c = ca + e + tp.off[q];
            in = in && c >= 0 && c < na;
          }
        }
        if (!in) a = T(0);
      }
      out[e] = a;
    }
    T* yp = y + s * ys + r;
    if (beta != T(0)) {
      T old[V];
      *reinterpret_cast<VT*>(old) = *reinterpret_cast<const VT*>(yp);
#pragma unroll
      for (int e = 0; e < V; ++e) out[e] = out[e] + beta * old[e];
    }
    *reinterpret_cast<VT*>(yp) = *reinterpret_cast<const VT*>(out);
  }
}

// LDS-tiled off-last-axis pass (round 4): a workgroup stages a (TA + reach) x 256-element block of rows
// along the pass axis once (16-B vector loads, zero outside the axis) and each thread sums its vector column
// for TA / 4 output rows from LDS (ds_read_b128 per tap): the vector kernel above re-reads every input row
// once per tap from L2.  Same sums in the same tap order, one fma each.
constexpr int kAxTA = 32, kAxTC = 256;  // output rows along the axis, elements along the inner dimension

template <typename T, bool ZERO_PARTIAL>
__global__ void __launch_bounds__(kBlock) axis_lds_kernel(int64_t sa, int64_t na, int64_t outer_per_stack,
                                                          AxisTaps<T> tp, int omin, int reach,
                                                          const T* __restrict__ x, int64_t xs, T* __restrict__ y,
                                                          int64_t ys, T beta) {
  constexpr int V = kVecN<T>;
  constexpr int TCV = kAxTC / 4;  // vectors per staged row (fp32: 64; fp64 rows are 128 elements wide)
  using VT = typename Vec4<T>::type;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  T* tile = reinterpret_cast<T*>(smem_raw);  // [row][TCV * V]
  constexpr int W = TCV * V;
  const int64_t oz = blockIdx.z;
  const int64_t s = oz / outer_per_stack, o = oz - s * outer_per_stack;
  const int64_t a0 = (int64_t)blockIdx.y * kAxTA;
  const int64_t c0 = (int64_t)blockIdx.x * W;  // first inner element of the block
  const int64_t base_x = s * xs + o * na * sa, base_y = s * ys + o * na * sa;
  const int rows = kAxTA + reach;
  for (int i = threadIdx.x; i < rows * TCV; i += kBlock) {
    const int r = i / TCV, cv = i - r * TCV;
    const int64_t ga = a0 + omin + r, gc = c0 + (int64_t)cv * V;
    T v[V];
    if (ga >= 0 && ga < na && gc < sa) {
      *reinterpret_cast<VT*>(v) = *reinterpret_cast<const VT*>(x + base_x + ga * sa + gc);
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) v[e] = T(0);
    }
    *reinterpret_cast<VT*>(tile + r * W + cv * V) = *reinterpret_cast<const VT*>(v);
  }
  __syncthreads();
  const int cv = (int)threadIdx.x % TCV, rg = (int)threadIdx.x / TCV;  // vector column, row group
  constexpr int RG = kBlock / TCV, RPT = kAxTA / RG;                      // row groups, rows per thread
  const int64_t gc = c0 + (int64_t)cv * V;
  if (gc >= sa) return;
#pragma unroll 1
  for (int k = 0; k < RPT; ++k) {
    const int i = rg * RPT + k;  // output row within the tile
    const int64_t ga = a0 + i;
    if (ga >= na) break;
    T acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = T(0);
    bool inside = true;
    for (int q = 0; q < tp.n; ++q) {
      const int o2 = tp.off[q];
      const int64_t c = ga + o2;
      if (c >= 0 && c < na) {
        T v[V];
        *reinterpret_cast<VT*>(v) = *reinterpret_cast<const VT*>(tile + (i + o2 - omin) * W + cv * V);
        const T cq = tp.coef[q];
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] = fma(cq, v[e], acc[e]);
      } else if (ZERO_PARTIAL) {
        inside = false;
      }
    }
    if (ZERO_PARTIAL && !inside) {
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] = T(0);
    }
    T* yp = y + base_y + ga * sa + gc;
    if (beta != T(0)) {
      T old[V];
      *reinterpret_cast<VT*>(old) = *reinterpret_cast<const VT*>(yp);
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] = acc[e] + beta * old[e];
    }
    *reinterpret_cast<VT*>(yp) = *reinterpret_cast<const VT*>(acc);
  }
}

template <typename T>
int launch_axis(int64_t stack, const Geom& g, int axis, int ntaps, const int32_t* offs, const double* coefs,
                int zero_partial, const void* x, int64_t xs, void* y, int64_t ys, double beta, hipStream_t s) {
  AxisTaps<T> tp;
  tp.n = ntaps;
  for (int q = 0; q < ntaps; ++q) {
    tp.off[q] = offs[q];
    tp.coef[q] = (T)coefs[q];
  }
  int64_t total = stack * g.size;
  constexpr int V = kVecN<T>;
  const bool last = axis == g.nd - 1;
  // off-last-axis passes LDS-tiled (512^3 Gaussian 1.78 -> 1.48 ms; PXA_TUNE_STENCIL_ND bit 2 turns it off,
  // bit 1 selects the scalar kernel for every pass)
  if ((tuning(PXA_TUNE_STENCIL_ND) & 6) == 0 && !last && g.n[g.nd - 1] % V == 0 && xs % V == 0 && ys % V == 0 &&
      aligned16(x) && aligned16(y) && ntaps > 0) {
    int omin = 0, omax = 0;
    for (int q = 0; q < ntaps; ++q) {
      omin = q == 0 || offs[q] < omin ? offs[q] : omin;
      omax = q == 0 || offs[q] > omax ? offs[q] : omax;
    }
    const int reach = omax - omin;
    const int64_t sa = g.st[axis], na = g.n[axis];
    const int64_t opv = g.size / (na * sa);
    const int W = (kAxTC / 4) * V;
    const size_t smem = (size_t)(kAxTA + reach) * W * sizeof(T);
    const int64_t gx = (sa + W - 1) / W, gy = (na + kAxTA - 1) / kAxTA, gz = stack * opv;
    if (smem <= 64 * 1024 && gy <= 65535 && gz <= 65535 && gx <= 0x7fffffff) {
      const dim3 grid((unsigned)gx, (unsigned)gy, (unsigned)gz);
      if (zero_partial)
        hipLaunchKernelGGL((axis_lds_kernel<T, true>), grid, dim3(kBlock), smem, s, sa, na, opv, tp, omin, reach,
                           (const T*)x, xs, (T*)y, ys, (T)beta);
      else
        hipLaunchKernelGGL((axis_lds_kernel<T, false>), grid, dim3(kBlock), smem, s, sa, na, opv, tp, omin, reach,
                           (const T*)x, xs, (T*)y, ys, (T)beta);
      return last_launch_status();
    }
  }
  if ((tuning(PXA_TUNE_STENCIL_ND) & 2) == 0 && g.n[g.nd - 1] % V == 0 && xs % V == 0 && ys % V == 0 &&
      aligned16(x) && aligned16(y)) {
    const int64_t items = total / V;
    auto launch = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(grid_for(items)), dim3(kBlock), 0, s, stack, g, axis, tp, (const T*)x, xs, (T*)y,
                         ys, (T)beta);
    };
    if (zero_partial) last ? launch(axis_vec_kernel<T, true, true>) : launch(axis_vec_kernel<T, true, false>);
    else last ? launch(axis_vec_kernel<T, false, true>) : launch(axis_vec_kernel<T, false, false>);
    return last_launch_status();
  }
  if (zero_partial)
    hipLaunchKernelGGL((axis_kernel<T, true>), dim3(grid_for(total)), dim3(kBlock), 0, s, stack, g, axis, tp,
                       (const T*)x, xs, (T*)y, ys, (T)beta);
  else
    hipLaunchKernelGGL((axis_kernel<T, false>), dim3(grid_for(total)), dim3(kBlock), 0, s, stack, g, axis, tp,
                       (const T*)x, xs, (T*)y, ys, (T)beta);
  return last_launch_status();
}

// ------------------------------------------------------------------ N-D stencil (device taps)
template <typename T, bool ZERO_PARTIAL>
__global__ void __launch_bounds__(kBlock) nd_kernel(int64_t stack, Geom g, int ntaps, const int32_t* __restrict__ offs,
                                                    const T* __restrict__ coefs, const T* __restrict__ x, int64_t xs,
                                                    T* __restrict__ y, int64_t ys, T beta) {
  const int64_t total = stack * g.size;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    int64_t s = t / g.size, r = t - s * g.size;
    int64_t c[PXA_MAX_DIM];
    int64_t rem = r;
#pragma unroll
    for (int d = 0; d < PXA_MAX_DIM; ++d) {
      if (d < g.nd) {
        c[d] = rem / g.st[d];
        rem -= c[d] * g.st[d];
      }
    }
    const T* xr = x + s * xs;
    T acc = T(0);
    bool inside = true;
    for (int q = 0; q < ntaps; ++q) {
      int64_t idx = 0;
      bool ok = true;
      for (int d = 0; d < g.nd; ++d) {
        int64_t cc = c[d] + offs[q * g.nd + d];
        ok = ok && (cc >= 0) && (cc < g.n[d]);
        idx += cc * g.st[d];
      }
      if (ok)
        acc = fma(coefs[q], xr[idx], acc);
      else if (ZERO_PARTIAL)
        inside = false;
    }
    if (ZERO_PARTIAL && !inside) acc = T(0);
    T* yp = y + s * ys + r;
    *yp = (beta == T(0)) ? acc : acc + beta * (*yp);
  }
}

// ------------------------------------------------------------------ N-D stencil, LDS-tiled (2-D / 3-D)
// One 256-thread workgroup per (4 RPT) x 64 output tile of one plane: the input box the taps reach (every
// plane of the axis-0 tap range for 3-D) is staged in LDS once, zero outside the array, and the tap table
// (staged-box offset, coefficient) beside it; a thread owns RPT rows of one column and, per tap, reads its
// RPT inputs at immediate offsets from one address (fixed pitch of 96 or 128: kernel widths up to 33 / 65).  Per output the taps are summed in list order with one fma each, so
// the result is the generic kernel's (which walks the same list) -- 15 x 15 taps on 2048^2: 2.08 ms there.
constexpr int kNdTX = 64;
constexpr int kNdMaxTaps = 2048;  // tap table in LDS: (offset, coefficient) per tap

struct BoxGeom {
  int nd;                      // 2 or 3
  int lo[3], hi[3];            // tap offset range per axis
  int np, rows;                // staged planes (3-D: hi0 - lo0 + 1) and rows (TY + hi_y - lo_y)
};

// RPT output rows per thread (TY = 4 RPT rows per tile), PITCH floats per staged row
template <typename T, bool ZP, int PITCH, int RPT>
__global__ void __launch_bounds__(kBlock) nd_tile_kernel(int64_t stack, Geom g, BoxGeom b, int ntaps,
                                                         const int32_t* __restrict__ offs,
                                                         const T* __restrict__ coefs, const T* __restrict__ x,
                                                         int64_t xs, T* __restrict__ y, int64_t ys, T beta) {
  constexpr int TY = 4 * RPT;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int nt4 = (ntaps + 3) & ~3;
  T* ctab = reinterpret_cast<T*>(smem_raw);          // coefficients
  int* otab = reinterpret_cast<int*>(ctab + nt4);    // staged-box offsets
  T* tile = reinterpret_cast<T*>(otab + nt4);
  const int nd = b.nd;
  const int ay = nd - 2, ax = nd - 1;
  const int64_t ny = g.n[ay], nx = g.n[ax];
  const int64_t n0 = nd == 3 ? g.n[0] : 1;
  const int64_t sp = blockIdx.z;  // stack * n0 + plane
  const int64_t s = sp / n0, p = sp - s * n0;
  const int y0 = (int)blockIdx.y * TY, x0 = (int)blockIdx.x * kNdTX;
  const T* xsb = x + s * xs;
  const int cols = kNdTX + b.hi[ax] - b.lo[ax];
  for (int q = threadIdx.x; q < ntaps; q += kBlock) {
    const int32_t* o = offs + q * nd;
    const int op = nd == 3 ? o[0] - b.lo[0] : 0;
    otab[q] = (op * b.rows + (o[ay] - b.lo[ay])) * PITCH + (o[ax] - b.lo[ax]);
    ctab[q] = coefs[q];
  }
  // stage the input box (zero outside the array)
  const int box = b.np * b.rows * cols;
  for (int i = threadIdx.x; i < box; i += kBlock) {
    const int pl = i / (b.rows * cols), rem = i - pl * (b.rows * cols);
    const int r = rem / cols, c = rem - r * cols;
    const int64_t gp = nd == 3 ? p + b.lo[0] + pl : 0;
    const int64_t gy = (int64_t)y0 + b.lo[ay] + r, gx = (int64_t)x0 + b.lo[ax] + c;
    T v = T(0);
    if (gp >= 0 && gp < n0 && gy >= 0 && gy < ny && gx >= 0 && gx < nx)
      v = xsb[(nd == 3 ? gp * g.st[0] : 0) + gy * g.st[ay] + gx];
    tile[(pl * b.rows + r) * PITCH + c] = v;
  }
  __syncthreads();
  const int col = (int)threadIdx.x % kNdTX, r0 = ((int)threadIdx.x / kNdTX) * RPT;
  const T* tb = tile + r0 * PITCH + col;
  T acc[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) acc[i] = T(0);
#pragma unroll 4
  for (int q = 0; q < ntaps; ++q) {
    const T cq = ctab[q];  // same address in every lane: broadcast
    const T* t = tb + otab[q];
#pragma unroll
    for (int i = 0; i < RPT; ++i) acc[i] = fma(cq, t[i * PITCH], acc[i]);
  }
  const int64_t gx = (int64_t)x0 + col;
  if (gx >= nx) return;
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int64_t gy = (int64_t)y0 + r0 + i;
    if (gy >= ny) continue;
    T v = acc[i];
    if (ZP) {  // every tap must lie inside the array
      bool in = gy + b.lo[ay] >= 0 && gy + b.hi[ay] < ny && gx + b.lo[ax] >= 0 && gx + b.hi[ax] < nx;
      if (nd == 3) in = in && p + b.lo[0] >= 0 && p + b.hi[0] < n0;
      if (!in) v = T(0);
    }
    T* yp = y + s * ys + (nd == 3 ? p * g.st[0] : 0) + gy * g.st[ay] + gx;
    *yp = (beta == T(0)) ? v : v + beta * (*yp);
  }
}

// the tiled kernel when it applies (2-D / 3-D, <= 2048 taps, kernel width <= 65, staged box <= 96 KB);
// false otherwise.  8 output rows per thread when the box fits, else 4.
template <typename T>
bool launch_nd_tile(int64_t stack, const Geom& g, int ntaps, const int32_t* offs, const T* coefs, const int32_t* lo,
                    const int32_t* hi, int zero_partial, const T* x, int64_t xs, T* y, int64_t ys, T beta,
                    hipStream_t st, int* status) {
  if ((g.nd != 2 && g.nd != 3) || lo == nullptr || hi == nullptr || ntaps < 1 || ntaps > kNdMaxTaps) return false;
  BoxGeom b;
  b.nd = g.nd;
  for (int a = 0; a < 3; ++a) b.lo[a] = b.hi[a] = 0;
  for (int a = 0; a < g.nd; ++a) {
    if (lo[a] > hi[a] || hi[a] - lo[a] > 64 || lo[a] < -65536 || hi[a] > 65536) return false;
    b.lo[a] = lo[a];
    b.hi[a] = hi[a];
  }
  const int ay = g.nd - 2, ax = g.nd - 1;
  const int width = b.hi[ax] - b.lo[ax] + 1;
  const int pitch = width <= 33 ? 96 : 128;
  b.np = g.nd == 3 ? b.hi[0] - b.lo[0] + 1 : 1;
  const size_t tabs = (size_t)((ntaps + 3) & ~3) * (sizeof(T) + sizeof(int));
  auto smem_for = [&](int ty) { return tabs + (size_t)b.np * (ty + b.hi[ay] - b.lo[ay]) * pitch * sizeof(T); };
  const int rpt = smem_for(32) <= 96 * 1024 ? 8 : 4;
  const int ty = 4 * rpt;
  b.rows = ty + b.hi[ay] - b.lo[ay];
  const size_t smem = smem_for(ty);
  if (smem > 96 * 1024) return false;
  const int64_t n0 = g.nd == 3 ? g.n[0] : 1;
  const int64_t tyn = (g.n[ay] + ty - 1) / ty, txn = (g.n[ax] + kNdTX - 1) / kNdTX;
  if (tyn > 65535 || txn > 0x7fffffff || stack * n0 > 0x7fffffff) return false;
  const dim3 grid((unsigned)txn, (unsigned)tyn, (unsigned)(stack * n0));
  static bool attr = false;
  if (!attr) {
    const void* ks[] = {(const void*)nd_tile_kernel<T, false, 96, 8>, (const void*)nd_tile_kernel<T, true, 96, 8>,
                        (const void*)nd_tile_kernel<T, false, 128, 8>, (const void*)nd_tile_kernel<T, true, 128, 8>,
                        (const void*)nd_tile_kernel<T, false, 96, 4>, (const void*)nd_tile_kernel<T, true, 96, 4>,
                        (const void*)nd_tile_kernel<T, false, 128, 4>, (const void*)nd_tile_kernel<T, true, 128, 4>};
    for (const void* k : ks) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    attr = true;
  }
  using K = void (*)(int64_t, Geom, BoxGeom, int, const int32_t*, const T*, const T*, int64_t, T*, int64_t, T);
  K kern;
  if (rpt == 8)
    kern = zero_partial ? (pitch == 96 ? nd_tile_kernel<T, true, 96, 8> : nd_tile_kernel<T, true, 128, 8>)
                        : (pitch == 96 ? nd_tile_kernel<T, false, 96, 8> : nd_tile_kernel<T, false, 128, 8>);
  else
    kern = zero_partial ? (pitch == 96 ? nd_tile_kernel<T, true, 96, 4> : nd_tile_kernel<T, true, 128, 4>)
                        : (pitch == 96 ? nd_tile_kernel<T, false, 96, 4> : nd_tile_kernel<T, false, 128, 4>);
  hipLaunchKernelGGL(kern, grid, dim3(kBlock), smem, st, stack, g, b, ntaps, offs, coefs, x, xs, y, ys, beta);
  *status = last_launch_status();
  return true;
}

// ------------------------------------------------------------------ Pad / Pad^T / Trim
struct PadGeom {
  Geom core;  // unpadded shape
  Geom pad;   // padded shape
  int64_t lo[PXA_MAX_DIM], hi[PXA_MAX_DIM];
  int mode[PXA_MAX_DIM];
};

// Map a padded coordinate j (0 <= j < n + lo + hi) to the core coordinate it copies
// (pad.py:254-304); returns -1 for constant-mode padding (value 0).
__device__ inline int64_t pad_src(int64_t j, int64_t n, int64_t lo, int mode) {
  int64_t c = j - lo;
  if (c >= 0 && c < n) return c;
  switch (mode) {
    case PXA_MODE_CONSTANT:
      return -1;
    case PXA_MODE_WRAP:
      return c < 0 ? c + n : c - n;
    case PXA_MODE_REFLECT:
      return c < 0 ? -c : 2 * (n - 1) - c;
    case PXA_MODE_SYMMETRIC:
      return c < 0 ? -c - 1 : 2 * n - 1 - c;
    default:  // edge
      return c < 0 ? 0 : n - 1;
  }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) pad_kernel(int64_t stack, PadGeom pg, const T* __restrict__ x,
                                                     T* __restrict__ y) {
  const int64_t total = stack * pg.pad.size;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    int64_t s = t / pg.pad.size, r = t - s * pg.pad.size;
    int64_t src = 0;
    bool zero = false;
    for (int d = 0; d < pg.pad.nd; ++d) {
      int64_t j = (r / pg.pad.st[d]) % pg.pad.n[d];
      int64_t c = pad_src(j, pg.core.n[d], pg.lo[d], pg.mode[d]);
      if (c < 0) zero = true;
      src += (c < 0 ? 0 : c) * pg.core.st[d];
    }
    y[t] = zero ? T(0) : x[s * pg.core.size + src];
  }
}

// Fold the pad region of axis `a` back onto the core of that axis (Pad^T for one axis, in place on
// a buffer whose axes < a are still padded and axes > a already folded... all strides given by
// `cur`).  One thread per element whose axis-a coordinate lies in the core.
template <typename T>
__global__ void __launch_bounds__(kBlock) fold_axis_kernel(int64_t stack, Geom cur, int a, int64_t n, int64_t lo,
                                                           int64_t hi, int mode, T* __restrict__ buf) {
  // iterate over all elements with axis-a coordinate in [lo, lo+n)
  Geom it = cur;
  it.n[a] = n;
  int64_t inner = 1;
  for (int d = 0; d < it.nd; ++d) inner *= it.n[d];
  const int64_t total = stack * inner;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    int64_t s = t / inner, r = t - s * inner;
    // unravel r over `it` shape
    int64_t off = 0, ca = 0;
    int64_t rem = r;
    for (int d = it.nd - 1; d >= 0; --d) {
      int64_t cd = rem % it.n[d];
      rem /= it.n[d];
      if (d == a) {
        ca = cd;
        cd += lo;
      }
      off += cd * cur.st[d];
    }
    T* base = buf + s * cur.size + off - (ca + lo) * cur.st[a];  // axis-a line start
    T v = base[(ca + lo) * cur.st[a]];
    // LHS images first, then RHS (pad.py:318-365 order).
    for (int64_t j = 0; j < lo; ++j)
      if (pad_src(j, n, lo, mode) == ca) v += base[j * cur.st[a]];
    for (int64_t j = lo + n; j < lo + n + hi; ++j)
      if (pad_src(j, n, lo, mode) == ca) v += base[j * cur.st[a]];
    base[(ca + lo) * cur.st[a]] = v;
  }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) trim_kernel(int64_t stack, PadGeom pg, int embed, const T* __restrict__ x,
                                                      T* __restrict__ y) {
  // embed = 0: y (core) <- x (padded) core window; embed = 1: y (padded) <- 0 | x (core)
  const Geom& big = pg.pad;
  const int64_t total = stack * (embed ? big.size : pg.core.size);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    if (embed) {
      int64_t s = t / big.size, r = t - s * big.size;
      int64_t src = 0;
      bool in = true;
      for (int d = 0; d < big.nd; ++d) {
        int64_t c = (r / big.st[d]) % big.n[d] - pg.lo[d];
        in = in && c >= 0 && c < pg.core.n[d];
        src += c * pg.core.st[d];
      }
      y[t] = in ? x[s * pg.core.size + src] : T(0);
    } else {
      int64_t s = t / pg.core.size, r = t - s * pg.core.size;
      int64_t dst = 0;
      for (int d = 0; d < big.nd; ++d) {
        int64_t c = (r / pg.core.st[d]) % pg.core.n[d] + pg.lo[d];
        dst += c * big.st[d];
      }
      y[t] = x[s * big.size + dst];
    }
  }
}

inline bool make_pad_geom(int ndim, const int64_t* shape, const int64_t* lo, const int64_t* hi, const int* modes,
                          PadGeom& pg) {
  if (!make_geom(ndim, shape, pg.core)) return false;
  int64_t ps[PXA_MAX_DIM];
  for (int d = 0; d < ndim; ++d) {
    if (lo[d] < 0 || hi[d] < 0) return false;
    ps[d] = shape[d] + lo[d] + hi[d];
    pg.lo[d] = lo[d];
    pg.hi[d] = hi[d];
    pg.mode[d] = modes ? modes[d] : PXA_MODE_CONSTANT;
    if (pg.mode[d] < 0 || pg.mode[d] > 4) return false;
    int64_t w = lo[d] > hi[d] ? lo[d] : hi[d];
    int64_t wmax = pg.mode[d] == PXA_MODE_WRAP || pg.mode[d] == PXA_MODE_SYMMETRIC ? shape[d]
                   : pg.mode[d] == PXA_MODE_REFLECT                                ? shape[d] - 1
                                                                                   : INT64_MAX;
    if (w > wmax) return false;  // pad.py:215-228
  }
  for (int d = ndim; d < PXA_MAX_DIM; ++d) {
    pg.lo[d] = pg.hi[d] = 0;
    pg.mode[d] = 0;
  }
  return make_geom(ndim, ps, pg.pad);
}

}  // namespace
}  // namespace pxa

using namespace pxa;

extern "C" {

int pxa_stencil_axis(int dtype, int64_t stack, int ndim, const int64_t* shape, int axis, int ntaps,
                     const int32_t* offsets, const double* coefs, int zero_partial, const void* x,
                     int64_t x_stack_stride, void* y, int64_t y_stack_stride, double beta, void* stream) {
  Geom g;
  PXA_CHECK_ARG(make_geom(ndim, shape, g));
  PXA_CHECK_ARG(axis >= 0 && axis < ndim && stack >= 0);
  PXA_CHECK_ARG(ntaps >= 0 && ntaps <= PXA_MAX_TAPS);
  PXA_CHECK_ARG(ntaps == 0 || (offsets != nullptr && coefs != nullptr));
  if (stack == 0) return PXA_OK;
  PXA_CHECK_ARG(x != nullptr && y != nullptr);
  PXA_DISPATCH(dtype, T,
               return launch_axis<T>(stack, g, axis, ntaps, offsets, coefs, zero_partial, x, x_stack_stride, y,
                                     y_stack_stride, beta, as_stream(stream)));
}

size_t pxa_stencil_sep_workspace_bytes(int dtype, int64_t stack, int ndim, const int64_t* shape, const int* ntaps) {
  Geom g;
  if (!make_geom(ndim, shape, g) || ntaps == nullptr) return 0;
  int k = 0;
  for (int d = 0; d < ndim; ++d) k += ntaps[d] > 0;
  size_t fields = k <= 1 ? 0 : (k == 2 ? 1 : 2);
  size_t es = dtype == PXA_F64 ? 8 : 4;
  return fields * (size_t)stack * (size_t)g.size * es;
}

int pxa_stencil_sep(int dtype, int64_t stack, int ndim, const int64_t* shape, const int* ntaps,
                    const int32_t* offsets, const double* coefs, const void* x, int64_t x_stack_stride, void* y,
                    int64_t y_stack_stride, double beta, void* work, void* stream) {
  Geom g;
  PXA_CHECK_ARG(make_geom(ndim, shape, g));
  PXA_CHECK_ARG(ntaps != nullptr && offsets != nullptr && coefs != nullptr);
  if (stack == 0) return PXA_OK;
  int axes[PXA_MAX_DIM], k = 0;
  for (int d = 0; d < ndim; ++d) {
    PXA_CHECK_ARG(ntaps[d] >= 0 && ntaps[d] <= PXA_MAX_TAPS);
    if (ntaps[d] > 0) axes[k++] = d;
  }
  hipStream_t s = as_stream(stream);
  size_t es = dtype == PXA_F64 ? 8 : 4;
  if (k == 0) {  // all-identity kernel: y = x + beta*y
    PXA_CHECK_ARG(x_stack_stride == g.size && y_stack_stride == g.size);
    return pxa_axpby(dtype, stack * g.size, 1.0, x, beta, beta == 0.0 ? nullptr : y, y, stream);
  }
  PXA_CHECK_ARG(k == 1 || work != nullptr);
  char* w0 = (char*)work;
  char* w1 = w0 + (size_t)stack * g.size * es;
  const void* src = x;
  int64_t srcs = x_stack_stride;
  for (int p = 0; p < k; ++p) {
    int a = axes[p];
    bool last = p == k - 1;
    void* dst = last ? y : (void*)((p % 2 == 0) ? w0 : w1);
    int64_t dsts = last ? y_stack_stride : g.size;
    int e;
    PXA_DISPATCH(dtype, T,
                 e = launch_axis<T>(stack, g, a, ntaps[a], offsets + a * PXA_MAX_TAPS, coefs + a * PXA_MAX_TAPS, 0,
                                    src, srcs, dst, dsts, last ? beta : 0.0, s));
    if (e) return e;
    src = dst;
    srcs = dsts;
  }
  return PXA_OK;
}

int pxa_stencil_nd(int dtype, int64_t stack, int ndim, const int64_t* shape, int ntaps, const int32_t* offsets_dev,
                   const void* coefs_dev, int zero_partial, const void* x, int64_t x_stack_stride, void* y,
                   int64_t y_stack_stride, double beta, void* stream) {
  Geom g;
  PXA_CHECK_ARG(make_geom(ndim, shape, g));
  PXA_CHECK_ARG(ntaps >= 0 && stack >= 0);
  PXA_CHECK_ARG(ntaps == 0 || (offsets_dev != nullptr && coefs_dev != nullptr));
  if (stack == 0) return PXA_OK;
  PXA_CHECK_ARG(x != nullptr && y != nullptr);
  int64_t total = stack * g.size;
  PXA_DISPATCH(dtype, T, {
    if (zero_partial)
      hipLaunchKernelGGL((nd_kernel<T, true>), dim3(grid_for(total)), dim3(kBlock), 0, as_stream(stream), stack, g,
                         ntaps, offsets_dev, (const T*)coefs_dev, (const T*)x, x_stack_stride, (T*)y, y_stack_stride,
                         (T)beta);
    else
      hipLaunchKernelGGL((nd_kernel<T, false>), dim3(grid_for(total)), dim3(kBlock), 0, as_stream(stream), stack, g,
                         ntaps, offsets_dev, (const T*)coefs_dev, (const T*)x, x_stack_stride, (T*)y, y_stack_stride,
                         (T)beta);
    return last_launch_status();
  });
}

int pxa_stencil_nd_box(int dtype, int64_t stack, int ndim, const int64_t* shape, int ntaps, const int32_t* offsets_dev,
                       const void* coefs_dev, const int32_t* off_lo, const int32_t* off_hi, int zero_partial,
                       const void* x, int64_t x_stack_stride, void* y, int64_t y_stack_stride, double beta,
                       void* stream) {
  Geom g;
  PXA_CHECK_ARG(make_geom(ndim, shape, g));
  PXA_CHECK_ARG(ntaps >= 0 && stack >= 0);
  PXA_CHECK_ARG(ntaps == 0 || (offsets_dev != nullptr && coefs_dev != nullptr));
  if (stack == 0) return PXA_OK;
  PXA_CHECK_ARG(x != nullptr && y != nullptr);
  if ((tuning(PXA_TUNE_STENCIL_ND) & 1) == 0) {
    PXA_DISPATCH(dtype, T, {
      int status = PXA_OK;
      if (launch_nd_tile<T>(stack, g, ntaps, offsets_dev, (const T*)coefs_dev, off_lo, off_hi, zero_partial,
                            (const T*)x, x_stack_stride, (T*)y, y_stack_stride, (T)beta, as_stream(stream), &status))
        return status;
    });
  }
  return pxa_stencil_nd(dtype, stack, ndim, shape, ntaps, offsets_dev, coefs_dev, zero_partial, x, x_stack_stride, y,
                        y_stack_stride, beta, stream);
}

int pxa_pad(int dtype, int64_t stack, int ndim, const int64_t* shape, const int64_t* pad_lo, const int64_t* pad_hi,
            const int* modes, const void* x, void* y, void* stream) {
  PadGeom pg;
  PXA_CHECK_ARG(pad_lo != nullptr && pad_hi != nullptr);
  PXA_CHECK_ARG(make_pad_geom(ndim, shape, pad_lo, pad_hi, modes, pg));
  if (stack == 0) return PXA_OK;
  PXA_CHECK_ARG(x != nullptr && y != nullptr);
  PXA_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((pad_kernel<T>), dim3(grid_for(stack * pg.pad.size)), dim3(kBlock), 0, as_stream(stream),
                       stack, pg, (const T*)x, (T*)y);
    return last_launch_status();
  });
}

int pxa_pad_adjoint(int dtype, int64_t stack, int ndim, const int64_t* shape, const int64_t* pad_lo,
                    const int64_t* pad_hi, const int* modes, const void* x, void* y, void* work, void* stream) {
  PadGeom pg;
  PXA_CHECK_ARG(pad_lo != nullptr && pad_hi != nullptr);
  PXA_CHECK_ARG(make_pad_geom(ndim, shape, pad_lo, pad_hi, modes, pg));
  if (stack == 0) return PXA_OK;
  PXA_CHECK_ARG(x != nullptr && y != nullptr && work != nullptr);
  hipStream_t s = as_stream(stream);
  size_t es = dtype == PXA_F64 ? 8 : 4;
  hipError_t me = hipMemcpyAsync(work, x, (size_t)stack * pg.pad.size * es, hipMemcpyDeviceToDevice, s);
  if (me) return (int)me;
  PXA_DISPATCH(dtype, T, {
    // Fold axes last -> first (pad.py:318-366), in place on `work` (padded layout throughout).
    for (int a = ndim - 1; a >= 0; --a) {
      if (pg.mode[a] == PXA_MODE_CONSTANT || (pg.lo[a] == 0 && pg.hi[a] == 0)) continue;
      int64_t items = stack * (pg.pad.size / pg.pad.n[a]) * pg.core.n[a];
      hipLaunchKernelGGL((fold_axis_kernel<T>), dim3(grid_for(items)), dim3(kBlock), 0, s, stack, pg.pad, a,
                         pg.core.n[a], pg.lo[a], pg.hi[a], pg.mode[a], (T*)work);
      int e = last_launch_status();
      if (e) return e;
    }
    hipLaunchKernelGGL((trim_kernel<T>), dim3(grid_for(stack * pg.core.size)), dim3(kBlock), 0, s, stack, pg, 0,
                       (const T*)work, (T*)y);
    return last_launch_status();
  });
}

int pxa_trim(int dtype, int64_t stack, int ndim, const int64_t* shape, const int64_t* lo, const int64_t* hi,
             int embed, const void* x, void* y, void* stream) {
  // `shape` is the PADDED (big) shape; the core is shape - lo - hi.
  PXA_CHECK_ARG(shape != nullptr && lo != nullptr && hi != nullptr && ndim >= 1 && ndim <= PXA_MAX_DIM);
  int64_t core[PXA_MAX_DIM];
  int modes[PXA_MAX_DIM] = {0, 0, 0, 0};
  for (int d = 0; d < ndim; ++d) {
    core[d] = shape[d] - lo[d] - hi[d];
    PXA_CHECK_ARG(core[d] >= 1);
  }
  PadGeom pg;
  PXA_CHECK_ARG(make_pad_geom(ndim, core, lo, hi, modes, pg));
  if (stack == 0) return PXA_OK;
  PXA_CHECK_ARG(x != nullptr && y != nullptr);
  int64_t total = stack * (embed ? pg.pad.size : pg.core.size);
  PXA_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((trim_kernel<T>), dim3(grid_for(total)), dim3(kBlock), 0, as_stream(stream), stack, pg,
                       embed, (const T*)x, (T*)y);
    return last_launch_status();
  });
}

}  // extern "C"
