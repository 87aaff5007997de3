// Fused primal-dual splitting iterations (PD3O, Condat-Vu) for TV-regularised deblurring of 2-D
// images and 3-D volumes: three launches per iteration instead of the reference's ~25 array passes.
//
// Problem:  f = 1/2 ||S . - y||^2 with S a separable zero-boundary
// stencil (Gaussian / Convolve / Stencil, operator/linop/stencil/stencil.py:441-461), K = Grad
// (forward differences over the D trailing axes, diff.py:1113-1265), h = lam L1 (anisotropic TV) or
// lam L21 over the D directions (isotropic TV), g in {None, PositiveOrthant, lam L1}.
//
// PD3O.m_step (opt/solver/pds.py:747-761):
//   x      = prox_g(u - tau K^T z)                            kernel A (with the axis-0 half of G x)
//   u_tmp  = x - tau grad f(x),  grad f(x) = G x - S^T y      kernel B (in-plane half of G x + update)
//   w      = x + u_tmp - u ;  u = (1 - rho) u + rho u_tmp     kernel B
//   z      = (1 - rho) z + rho fenchel_prox_h(z + sigma K w)  kernel C
// CondatVu.m_step (pds.py:429-442):
//   x_tmp  = prox_g(x - tau grad f(x) - tau K^T z)            kernels A (axis 0 of G x) + B
//   w      = 2 x_tmp - x ;  x = rho x_tmp + (1 - rho) x       kernel B
//   z      = rho fenchel_prox_h(z + sigma K w) + (1 - rho) z  kernel C
//
// G = S^T S is separable: G = G0 (x) G1 (x) G2 with G_a = H_a^T H_a (H_a the zero-boundary 1-D
// correlation of axis a), so G x is evaluated as G12 (G0 x):
//  * kernel A marches each pixel column along axis 0 and keeps the H0 and H0^T windows in two
//    register rings (2 R0 + 1 planes each): the plain two-pass form, exact at the boundary planes,
//    one HBM read of the input per voxel.  PD3O builds its input x = prox_g(u - tau K^T z) on the fly
//    (and stores it: x is the iterate the solver returns); Condat-Vu reads x.
//  * kernel B is the LDS-tiled in-plane normal-operator sweep of pgd_tv2d.hip (tile2d.hpp: two
//    register-blocked 4R+1-tap passes with exact boundary-row corrections) over every plane, with the
//    solver's point-wise update fused into its epilogue.
//  * kernel C is the dual update: K w (one forward neighbour per direction, from cache), fenchel_prox
//    (operator.py:905-944) as the projection onto the lam-ball of the dual norm that its Moreau form
//    equals (pds3d.hpp dual_out), and the relaxation.
//  * pxa_pds_step_la replaces kernels C and A by kernel D (pds_march.hpp): the dual update of iteration k
//    fused with the axis-0 march of iteration k + 1, two launches per iteration.
// Compulsory HBM traffic per voxel (fp32): PD3O A 24 B + B 24 B + C 28 B = 76 B (80 B);
// Condat-Vu A 8 B + B 32 B + C 28 B = 68 B (SURVEY: 68 B).
//
// Parity: the step follows the reference's arithmetic per voxel except that G x replaces
// S^T (S x - y) + ... (same operator, different fp32 rounding order: see pgd_tv2d.hip).
#include <atomic>
#include <map>
#include <mutex>

#include "pds_march.hpp"

namespace pxa {
namespace pds {

// kernel D's soft-coupling counters (pds_march.hpp): per device, grown on demand, zeroed once
unsigned* progress_counters(int64_t units) {
  static std::mutex mu;
  static std::map<int, std::pair<unsigned*, int64_t>> bufs;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  auto& b = bufs[dev];
  if (b.second < units) {
    unsigned* p = nullptr;
    if (hipMalloc((void**)&p, (size_t)units * sizeof(unsigned)) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, (size_t)units * sizeof(unsigned)) != hipSuccess) return nullptr;
    // (the previous, smaller buffer stays allocated: a kernel still in flight may use it)
    b = {p, units};
  }
  return b.first;
}

unsigned next_progress_tag() {
  static std::atomic<unsigned> n{0};
  return ((n.fetch_add(1) % 65535u) + 1u) << 16;
}

// ------------------------------------------------------------------ kernel C: dual update
template <typename T>
struct PdsC {
  PdsGeom<T> g;
  T sigma, lam, rho, omr;
  int seg;               // planes per axis-0 segment
};

template <typename T, int NV>
__device__ inline void ldv(const T* p, T (&v)[NV]) {
  if constexpr (NV == kVecN<T>)
    *reinterpret_cast<typename Vec4<T>::type*>(v) = *reinterpret_cast<const typename Vec4<T>::type*>(p);
  else
    v[0] = p[0];
}

// Thread = NV consecutive in-plane positions of one row; it marches the planes of its segment, so the
// axis-0 forward neighbour w(p + 1) is loaded once and carried to the next step.  The in-plane block
// index is XCD-banded (tile2d::xcd_tile) so that the row+1 neighbour is usually read from the L2 of the
// same XCD, where the neighbouring block marches in step.
// PF (the default; PXA_TUNE_DUAL_ROWS = 1 turns it off): z and the row + 1 / column + 1 neighbours of plane p + 1 are
// loaded while plane p is computed (two planes of loads in flight per thread); the same values in the same expressions:
// the same bits.
template <typename T, int NV, bool ISO, bool PD3O, bool NT, bool PF = false>
__global__ void __launch_bounds__(kBlock) pds_dual_kernel(PdsC<T> p, const T* __restrict__ w,
                                                          const T* __restrict__ z, T* __restrict__ zo) {
  const PdsGeom<T> g = p.g;
  const T sigma = p.sigma, lam = p.lam, rho = p.rho, omr = p.omr;
  const int n0 = g.n0, n1 = g.n1, n2 = g.n2, D = g.D;
  const int64_t M = (int64_t)n1 * n2, N = M * n0;
  const int a_first = 3 - D;
  const unsigned blk = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t j0 = ((int64_t)blk * kBlock + threadIdx.x) * NV;
  if (j0 >= M) return;  // no barriers below
  const int r = (int)(j0 / n2), c = (int)(j0 - (int64_t)r * n2);
  const int64_t s = blockIdx.z;
  const int pb = blockIdx.y * p.seg;
  const int pe = pb + p.seg < n0 ? pb + p.seg : n0;
  const T* ws = w + s * N + j0;
  const T* zs = z + s * (int64_t)D * N + j0;
  T* zos = zo + s * (int64_t)D * N + j0;
  const bool row_nb = r + 1 < n1, col_nb = c + NV < n2;
  T wn0[NV];  // w at the current plane (carried from the previous step)
  ldv<T, NV>(ws + (int64_t)pb * M, wn0);
  // PF: the next plane's z, w row + 1 and w column + 1 (the loads below, one plane early)
  T fz[3][NV], fr[NV], fcol;
  auto fetch = [&](int pl) {
    const int64_t off = (int64_t)pl * M;
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
      if (ax < a_first) continue;
      if (NT)
        ldn_nt<T, NV>(zs + (int64_t)(ax - a_first) * N + off, fz[ax]);
      else
        ldv<T, NV>(zs + (int64_t)(ax - a_first) * N + off, fz[ax]);
    }
    if (row_nb) {
      ldv<T, NV>(ws + off + n2, fr);
    } else {
#pragma unroll
      for (int e = 0; e < NV; ++e) fr[e] = T(0);
    }
    fcol = col_nb ? ws[off + NV] : T(0);
  };
  if (PF) fetch(pb);
  for (int pl = pb; pl < pe; ++pl) {
    const int64_t off = (int64_t)pl * M;
    T wc[NV], wp[NV];
#pragma unroll
    for (int e = 0; e < NV; ++e) wc[e] = wn0[e];
    if (pl + 1 < n0) {
      ldv<T, NV>(ws + off + M, wp);
    } else {
#pragma unroll
      for (int e = 0; e < NV; ++e) wp[e] = T(0);
    }
    T cz[3][NV], cr[NV], ccol = T(0);
    if (PF) {
#pragma unroll
      for (int ax = 0; ax < 3; ++ax)
#pragma unroll
        for (int e = 0; e < NV; ++e) cz[ax][e] = fz[ax][e];
#pragma unroll
      for (int e = 0; e < NV; ++e) cr[e] = fr[e];
      ccol = fcol;
      if (pl + 1 < pe) fetch(pl + 1);
    }
    T zin[3][NV], zc[3][NV];
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
      if (ax < a_first) continue;
      T wn[NV];
      if (ax == 0) {
#pragma unroll
        for (int e = 0; e < NV; ++e) wn[e] = wp[e];
      } else if (ax == 1) {
        if (PF) {
#pragma unroll
          for (int e = 0; e < NV; ++e) wn[e] = cr[e];
        } else if (row_nb) {
          ldv<T, NV>(ws + off + n2, wn);
        } else {
#pragma unroll
          for (int e = 0; e < NV; ++e) wn[e] = T(0);
        }
      } else {
#pragma unroll
        for (int e = 0; e + 1 < NV; ++e) wn[e] = wc[e + 1];
        wn[NV - 1] = PF ? ccol : (col_nb ? ws[off + NV] : T(0));
      }
      if (PF) {
#pragma unroll
        for (int e = 0; e < NV; ++e) zc[ax][e] = cz[ax][e];
      } else if (NT)
        ldn_nt<T, NV>(zs + (int64_t)(ax - a_first) * N + off, zc[ax]);
      else
        ldv<T, NV>(zs + (int64_t)(ax - a_first) * N + off, zc[ax]);
#pragma unroll
      for (int e = 0; e < NV; ++e) zin[ax][e] = dual_in<T>(zc[ax][e], wc[e], wn[e], g.c0[ax], g.c1[ax], sigma);
    }
#pragma unroll
    for (int e = 0; e < NV; ++e) wn0[e] = wp[e];
    T zo3[3][NV];
#pragma unroll
    for (int e = 0; e < NV; ++e) {
      T zc1[3], zi1[3], zn1[3];
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) {
        zc1[ax] = ax < a_first ? T(0) : zc[ax][e];
        zi1[ax] = ax < a_first ? T(0) : zin[ax][e];
      }
      dual_out<T, ISO, PD3O>(zc1, zi1, a_first, lam, rho, omr, zn1);
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) zo3[ax][e] = zn1[ax];
    }
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
      if (ax < a_first) continue;
      T zn[NV];
#pragma unroll
      for (int e = 0; e < NV; ++e) zn[e] = zo3[ax][e];
      T* zq = zos + (int64_t)(ax - a_first) * N + off;
      if (NT)
        stn_nt<T, NV>(zq, zn);
      else if constexpr (NV == kVecN<T>)
        *reinterpret_cast<typename Vec4<T>::type*>(zq) = *reinterpret_cast<const typename Vec4<T>::type*>(zn);
      else
        zq[0] = zn[0];
    }
  }
}

// Row-blocked form (RB >= 2 rows per thread): a thread owns NV positions of RB consecutive rows, so the row + 1
// neighbour of every row but its last is its own next row (already in registers at this plane) and only one
// neighbour row per RB rows is read from another thread's rows: w is read 1 + 1 / RB times per voxel instead of
// twice, and the HBM over-fetch of the neighbour rows that another workgroup has not kept in L2 shrinks with it
// (1024^3: 1.107 x compulsory with RB = 1; profiles/r06*_k4_rows.txt).  Same per-element expressions: the same bits.
template <typename T, int NV, int RB, bool ISO, bool PD3O, bool NT>
__global__ void __launch_bounds__(kBlock) pds_dual_rows_kernel(PdsC<T> p, const T* __restrict__ w,
                                                               const T* __restrict__ z, T* __restrict__ zo) {
  const PdsGeom<T> g = p.g;
  const T sigma = p.sigma, lam = p.lam, rho = p.rho, omr = p.omr;
  const int n0 = g.n0, n1 = g.n1, n2 = g.n2, D = g.D;
  const int64_t M = (int64_t)n1 * n2, N = M * n0;
  const int a_first = 3 - D;
  const int cgs = (n2 + NV - 1) / NV;  // column groups per row
  const unsigned blk = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t t = (int64_t)blk * kBlock + threadIdx.x;
  const int64_t rg = t / cgs;
  if (rg * RB >= n1) return;  // no barriers below
  const int r = (int)(rg * RB), c = (int)(t - rg * cgs) * NV;
  const int nr = n1 - r < RB ? n1 - r : RB;  // rows of this thread inside the plane
  const int64_t s = blockIdx.z;
  const int pb = blockIdx.y * p.seg;
  const int pe = pb + p.seg < n0 ? pb + p.seg : n0;
  const int64_t j0 = (int64_t)r * n2 + c;
  const T* ws = w + s * N + j0;
  const T* zs = z + s * (int64_t)D * N + j0;
  T* zos = zo + s * (int64_t)D * N + j0;
  const bool row_nb = r + RB < n1, col_nb = c + NV < n2;
  T wcur[RB][NV];  // w at the current plane, rows r .. r + RB - 1 (carried from the previous step)
#pragma unroll
  for (int i = 0; i < RB; ++i) {
    if (i < nr) {
      ldv<T, NV>(ws + (int64_t)pb * M + (int64_t)i * n2, wcur[i]);
    } else {
#pragma unroll
      for (int e = 0; e < NV; ++e) wcur[i][e] = T(0);
    }
  }
  for (int pl = pb; pl < pe; ++pl) {
    const int64_t off = (int64_t)pl * M;
    T wnext[RB][NV], wrow[NV];
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      if (pl + 1 < n0 && i < nr) {
        ldv<T, NV>(ws + off + M + (int64_t)i * n2, wnext[i]);
      } else {
#pragma unroll
        for (int e = 0; e < NV; ++e) wnext[i][e] = T(0);
      }
    }
    if (row_nb) {
      ldv<T, NV>(ws + off + (int64_t)RB * n2, wrow);
    } else {
#pragma unroll
      for (int e = 0; e < NV; ++e) wrow[e] = T(0);
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      if (i >= nr) continue;
      const int64_t ro = off + (int64_t)i * n2;
      T zin[3][NV], zc[3][NV];
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) {
        if (ax < a_first) continue;
        T wn[NV];
        if (ax == 0) {
#pragma unroll
          for (int e = 0; e < NV; ++e) wn[e] = wnext[i][e];
        } else if (ax == 1) {
#pragma unroll
          for (int e = 0; e < NV; ++e) wn[e] = i + 1 < RB ? wcur[i + 1 < RB ? i + 1 : i][e] : wrow[e];
          if (i + 1 < RB && i + 1 >= nr) {  // the plane's last row inside this thread's block: zero neighbour
#pragma unroll
            for (int e = 0; e < NV; ++e) wn[e] = T(0);
          }
        } else {
#pragma unroll
          for (int e = 0; e + 1 < NV; ++e) wn[e] = wcur[i][e + 1];
          wn[NV - 1] = col_nb ? ws[ro + NV] : T(0);
        }
        if (NT)
          ldn_nt<T, NV>(zs + (int64_t)(ax - a_first) * N + ro, zc[ax]);
        else
          ldv<T, NV>(zs + (int64_t)(ax - a_first) * N + ro, zc[ax]);
#pragma unroll
        for (int e = 0; e < NV; ++e) zin[ax][e] = dual_in<T>(zc[ax][e], wcur[i][e], wn[e], g.c0[ax], g.c1[ax], sigma);
      }
      T zo3[3][NV];
#pragma unroll
      for (int e = 0; e < NV; ++e) {
        T zc1[3], zi1[3], zn1[3];
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {
          zc1[ax] = ax < a_first ? T(0) : zc[ax][e];
          zi1[ax] = ax < a_first ? T(0) : zin[ax][e];
        }
        dual_out<T, ISO, PD3O>(zc1, zi1, a_first, lam, rho, omr, zn1);
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) zo3[ax][e] = zn1[ax];
      }
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) {
        if (ax < a_first) continue;
        T zn[NV];
#pragma unroll
        for (int e = 0; e < NV; ++e) zn[e] = zo3[ax][e];
        T* zq = zos + (int64_t)(ax - a_first) * N + ro;
        if (NT)
          stn_nt<T, NV>(zq, zn);
        else if constexpr (NV == kVecN<T>)
          *reinterpret_cast<typename Vec4<T>::type*>(zq) = *reinterpret_cast<const typename Vec4<T>::type*>(zn);
        else
          zq[0] = zn[0];
      }
    }
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
      for (int e = 0; e < NV; ++e) wcur[i][e] = wnext[i][e];
  }
}

// Plane-block form (3-D, 16-B vectors; PXA_TUNE_DUAL_ROWS = 8): a workgroup owns a block of kLdsRB rows x kLdsC columns
// of the plane and marches its axis-0 segment; at each plane every thread stores its own w vector into an LDS image
// of the block (double-buffered by plane parity), the block's halo -- the row below it and the column right of it,
// fetched one plane ahead -- goes in beside it, and the row + 1 / column + 1 neighbours are read from LDS: a w row is
// fetched from memory by its own workgroup only, plus once more as the halo of the block above it (1 + 1 / kLdsRB
// reads per voxel instead of up to 2 with the one-row kernel, whose neighbour rows other workgroups fetch at their
// own pace).  One barrier per plane.  Same per-element expressions: the same bits.
constexpr int kLdsRB = 8;    // rows per block
constexpr int kLdsC = 128;   // columns per block (32 threads x 4)
constexpr int kLdsP = kLdsC + 4;  // LDS pitch (floats): the halo column's vector at kLdsC

template <bool ISO, bool PD3O, bool ZA>
__global__ void __launch_bounds__(kBlock) pds_dual_lds_kernel(PdsC<float> p, const float* __restrict__ w,
                                                              const float* __restrict__ z, float* __restrict__ zo,
                                                              int tiles2) {
  static_assert(kBlock == kLdsRB * kLdsC / 4, "one 4-vector per thread");
  __shared__ __align__(16) float img[2][kLdsRB + 1][kLdsP];
  const PdsGeom<float> g = p.g;
  const float sigma = p.sigma, lam = p.lam, rho = p.rho, omr = p.omr;
  const int n0 = g.n0, n1 = g.n1, n2 = g.n2;
  const int64_t M = (int64_t)n1 * n2, N = M * n0;
  const unsigned blk = xcd_tile(blockIdx.x, gridDim.x);
  const int tr = (int)(blk / (unsigned)tiles2), tc = (int)(blk - (unsigned)tr * (unsigned)tiles2);
  const int t = threadIdx.x, lr = t >> 5, lc = 4 * (t & 31);
  const int r = tr * kLdsRB + lr, c = tc * kLdsC + lc;
  const bool live = r < n1 && c < n2;  // (n2 % 4 == 0: a vector is wholly inside or outside)
  const int64_t s = blockIdx.z;
  const int pb = blockIdx.y * p.seg;
  const int pe = pb + p.seg < n0 ? pb + p.seg : n0;
  const int64_t j0 = (int64_t)r * n2 + c;
  const float* wb = w + s * N;
  const float* zs = z + s * (int64_t)3 * N + j0;
  float* zos = zo + s * (int64_t)3 * N + j0;
  // halo lanes: threads 0..31 the row below the block (4 columns each), 32..39 the column right of it (one row each)
  const int hr = tr * kLdsRB + kLdsRB, hc = tc * kLdsC + lc;        // row halo position (t < 32)
  const int vr = tr * kLdsRB + (t - 32), vc = tc * kLdsC + kLdsC;   // column halo position (32 <= t < 40)
  const bool hrow = t < 32, hcol = t >= 32 && t < 32 + kLdsRB;
  const bool hin = hrow ? (hr < n1 && hc < n2) : hcol ? (vr < n1 && vc < n2) : false;
  const int64_t hoff = hrow ? (int64_t)hr * n2 + hc : (int64_t)vr * n2 + vc;
  auto load_w = [&](int pl, float (&v)[4]) {
    if (live && pl < n0) {
      ldv<float, 4>(wb + (int64_t)pl * M + j0, v);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = 0.f;
    }
  };
  auto load_h = [&](int pl, float (&v)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = 0.f;
    if (hin && pl < n0) {
      if (hrow)
        ldv<float, 4>(wb + (int64_t)pl * M + hoff, v);
      else
        v[0] = wb[(int64_t)pl * M + hoff];
    }
  };
  float wc[4], wp[4], hc4[4], hn4[4];
  load_w(pb, wc);
  load_h(pb, hc4);
  float zn[3][4];  // z of the next plane (ZA: loaded one plane ahead)
  auto load_z = [&](int pl, float (&v)[3][4]) {
    if (live && pl < pe) {
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) ldn_nt<float, 4>(zs + (int64_t)ax * N + (int64_t)pl * M, v[ax]);
    }
  };
  if (ZA) load_z(pb, zn);
  for (int pl = pb; pl < pe; ++pl) {
    const int par = pl & 1;
    const int64_t off = (int64_t)pl * M;
    float zc[3][4];
    if (ZA) {
#pragma unroll
      for (int ax = 0; ax < 3; ++ax)
#pragma unroll
        for (int e = 0; e < 4; ++e) zc[ax][e] = zn[ax][e];
    }
    load_w(pl + 1, wp);  // next plane: own vector and halo, in flight through this plane
    load_h(pl + 1, hn4);
    if (ZA)
      load_z(pl + 1, zn);
    else
      load_z(pl, zc);
    // this plane's w image: own vectors, the halo row / column (zeros outside the image)
    *reinterpret_cast<float4*>(&img[par][lr][lc]) = make_float4(wc[0], wc[1], wc[2], wc[3]);
    if (hrow) *reinterpret_cast<float4*>(&img[par][kLdsRB][lc]) = make_float4(hc4[0], hc4[1], hc4[2], hc4[3]);
    if (hcol) img[par][t - 32][kLdsC] = hc4[0];
    __syncthreads();  // (double buffer: the next plane writes the other image, so one barrier per plane)
    if (live) {
      float wr[4];
      const float4 q = *reinterpret_cast<const float4*>(&img[par][lr + 1][lc]);
      wr[0] = q.x, wr[1] = q.y, wr[2] = q.z, wr[3] = q.w;
      const float wcol = img[par][lr][lc + 4];
      float zin[3][4];
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) {
        float wn[4];
        if (ax == 0) {
#pragma unroll
          for (int e = 0; e < 4; ++e) wn[e] = wp[e];
        } else if (ax == 1) {
#pragma unroll
          for (int e = 0; e < 4; ++e) wn[e] = r + 1 < n1 ? wr[e] : 0.f;
        } else {
#pragma unroll
          for (int e = 0; e < 3; ++e) wn[e] = wc[e + 1];
          wn[3] = c + 4 < n2 ? wcol : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) zin[ax][e] = dual_in<float>(zc[ax][e], wc[e], wn[e], g.c0[ax], g.c1[ax], sigma);
      }
      float zo3[3][4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float zc1[3], zi1[3], zn1[3];
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {
          zc1[ax] = zc[ax][e];
          zi1[ax] = zin[ax][e];
        }
        dual_out<float, ISO, PD3O>(zc1, zi1, 0, lam, rho, omr, zn1);
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) zo3[ax][e] = zn1[ax];
      }
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) stn_nt<float, 4>(zos + (int64_t)ax * N + off, zo3[ax]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      wc[e] = wp[e];
      hc4[e] = hn4[e];
    }
  }
}

template <bool PD3O, bool ZA>
int launch_c_lds(const PdsC<float>& pc, bool iso, int nseg, const void* w, const void* z, void* zo, hipStream_t st) {
  const int tiles1 = (pc.g.n1 + kLdsRB - 1) / kLdsRB, tiles2 = (pc.g.n2 + kLdsC - 1) / kLdsC;
  dim3 grid((unsigned)((int64_t)tiles1 * tiles2), (unsigned)nseg, (unsigned)pc.g.stack);
  if (iso)
    hipLaunchKernelGGL((pds_dual_lds_kernel<true, PD3O, ZA>), grid, dim3(kBlock), 0, st, pc, (const float*)w, (const float*)z,
                       (float*)zo, tiles2);
  else
    hipLaunchKernelGGL((pds_dual_lds_kernel<false, PD3O, ZA>), grid, dim3(kBlock), 0, st, pc, (const float*)w, (const float*)z,
                       (float*)zo, tiles2);
  return last_launch_status();
}

template <typename T, int NV, int RB, bool PD3O>
int launch_c_rows(const PdsC<T>& pc, bool iso, int nseg, const void* w, const void* z, void* zo, hipStream_t st) {
  const int64_t items = (int64_t)((pc.g.n1 + RB - 1) / RB) * ((pc.g.n2 + NV - 1) / NV);
  const int64_t blocks = (items + kBlock - 1) / kBlock;
  dim3 grid((unsigned)blocks, (unsigned)nseg, (unsigned)pc.g.stack);
  if (iso)
    hipLaunchKernelGGL((pds_dual_rows_kernel<T, NV, RB, true, PD3O, true>), grid, dim3(kBlock), 0, st, pc, (const T*)w,
                       (const T*)z, (T*)zo);
  else
    hipLaunchKernelGGL((pds_dual_rows_kernel<T, NV, RB, false, PD3O, true>), grid, dim3(kBlock), 0, st, pc, (const T*)w,
                       (const T*)z, (T*)zo);
  return last_launch_status();
}

template <typename T, int NV, bool PD3O>
int launch_c(const PdsC<T>& pc, bool iso, int64_t M, int nseg, const void* w, const void* z, void* zo,
             hipStream_t st) {
  // rows per thread (PXA_TUNE_DUAL_ROWS): 1 the one-row kernel, 2 / 4 the row-blocked kernel
  const int64_t rb = tuning(PXA_TUNE_DUAL_ROWS);
  if constexpr (sizeof(T) == 4 && NV == 4) {
    if (rb == 8 && pc.g.D == 3) return launch_c_lds<PD3O, false>(pc, iso, nseg, w, z, zo, st);
    if (rb == 9 && pc.g.D == 3) return launch_c_lds<PD3O, true>(pc, iso, nseg, w, z, zo, st);
  }
  if (rb == 2) return launch_c_rows<T, NV, 2, PD3O>(pc, iso, nseg, w, z, zo, st);
  if (rb == 4) return launch_c_rows<T, NV, 4, PD3O>(pc, iso, nseg, w, z, zo, st);
  const int64_t blocks = (M + (int64_t)kBlock * NV - 1) / ((int64_t)kBlock * NV);
  dim3 grid((unsigned)blocks, (unsigned)nseg, (unsigned)pc.g.stack);
  // z / z_out non-temporal (read / written once): w's row + 1 neighbours stay in L2 (1024^3, r04b: fetch 22.5
  // -> 19 B/voxel, 5.9 -> 5.1-5.7 ms)
  if (rb != 1) {  // the next plane's loads one plane early (default; 1: without, A/B -- 1024^3 r06ar: 5.00 -> 4.94 ms)
    if (iso)
      hipLaunchKernelGGL((pds_dual_kernel<T, NV, true, PD3O, true, true>), grid, dim3(kBlock), 0, st, pc, (const T*)w,
                         (const T*)z, (T*)zo);
    else
      hipLaunchKernelGGL((pds_dual_kernel<T, NV, false, PD3O, true, true>), grid, dim3(kBlock), 0, st, pc, (const T*)w,
                         (const T*)z, (T*)zo);
    return last_launch_status();
  }
  if (iso)
    hipLaunchKernelGGL((pds_dual_kernel<T, NV, true, PD3O, true>), grid, dim3(kBlock), 0, st, pc, (const T*)w,
                       (const T*)z, (T*)zo);
  else
    hipLaunchKernelGGL((pds_dual_kernel<T, NV, false, PD3O, true>), grid, dim3(kBlock), 0, st, pc, (const T*)w,
                       (const T*)z, (T*)zo);
  return last_launch_status();
}

// Kernel C over a whole (stack, n0, n1, n2) geometry: z_out = relax(fenchel_prox_h(z + sigma K w)).  The
// march is split into axis-0 segments so that about 2048 workgroups are in flight (no halo: w(p + 1) is a
// plain load; at 1024^3 2048 took 5.0-5.1 ms against 5.1-5.7 ms at 4096, profiles/r04_k4_wgs.txt).  pd3o selects the relaxation order: (1 - rho) z + rho z_t, else rho z_t + (1 - rho) z.
template <typename T>
int run_c(const PdsGeom<T>& g, T sigma, T lam, T rho, T omr, bool pd3o, bool iso, const void* w, const void* z,
          void* z_out, hipStream_t st) {
  constexpr int V = kVecN<T>;
  const int64_t M = (int64_t)g.n1 * g.n2;
  PdsC<T> pc;
  pc.g = g;
  pc.sigma = sigma;
  pc.lam = lam;
  pc.rho = rho;
  pc.omr = omr;
  const bool vec = (g.n2 % V == 0) && aligned16(w) && aligned16(z) && aligned16(z_out);
  const int nv = vec ? V : 1;
  const int64_t rbt = tuning(PXA_TUNE_DUAL_ROWS);
  const int64_t rbk = rbt == 2 ? 2 : rbt == 4 ? 4 : 1;
  int64_t blocks = g.stack * ((M + (int64_t)kBlock * nv * rbk - 1) / ((int64_t)kBlock * nv * rbk));
  if ((rbt == 8 || rbt == 9) && vec && g.D == 3 && sizeof(T) == 4)  // (the plane-block kernel's block count)
    blocks = g.stack * (int64_t)((g.n1 + kLdsRB - 1) / kLdsRB) * ((g.n2 + kLdsC - 1) / kLdsC);
  const int64_t target = tuning(PXA_TUNE_DUAL_WGS) > 0 ? tuning(PXA_TUNE_DUAL_WGS) : 2048;  // A/B knob
  int cseg = (int)((target + blocks - 1) / blocks);
  if (cseg > g.n0) cseg = g.n0;
  if (cseg < 1) cseg = 1;
  pc.seg = (int)((g.n0 + cseg - 1) / cseg);
  cseg = (int)((g.n0 + pc.seg - 1) / pc.seg);
  if (vec)
    return pd3o ? launch_c<T, V, true>(pc, iso, M, cseg, w, z, z_out, st) : launch_c<T, V, false>(pc, iso, M, cseg, w, z, z_out, st);
  return pd3o ? launch_c<T, 1, true>(pc, iso, M, cseg, w, z, z_out, st) : launch_c<T, 1, false>(pc, iso, M, cseg, w, z, z_out, st);
}

// pxa_tv_dual_update: kernel C alone (the "Gradient + prox" kernel of SURVEY §8(d), K4)
template <typename T>
int dual_entry(int relax, const int64_t* geom, const double* diff, double sigma, double lam, double rho, int h_kind,
               const void* w, const void* z, void* z_out, hipStream_t st) {
  PXA_CHECK_ARG(geom && diff && w && z && z_out && z_out != w);
  PXA_CHECK_ARG(relax == 0 || relax == 1);
  PXA_CHECK_ARG(h_kind == 0 || h_kind == 1);
  const int64_t stack = geom[0], n0 = geom[1], n1 = geom[2], n2 = geom[3], D = geom[4];
  PXA_CHECK_ARG(stack >= 1 && stack <= 65535 && n0 >= 1 && n1 >= 1 && n2 >= 1);
  PXA_CHECK_ARG(n0 <= 0x7fffffff && n1 <= 0x7fffffff && n2 <= 0x7fffffff && n0 * n1 * n2 <= ((int64_t)1 << 40));
  PXA_CHECK_ARG(D == 2 || D == 3);
  PXA_CHECK_ARG(D == 3 || n0 == 1);
  PdsGeom<T> g;
  g.stack = stack;
  g.y_images = 1;
  g.n0 = (int)n0;
  g.n1 = (int)n1;
  g.n2 = (int)n2;
  g.D = (int)D;
  for (int a = 0; a < 3; ++a) {
    g.c0[a] = (T)diff[a];
    g.c1[a] = (T)diff[3 + a];
  }
  return run_c<T>(g, (T)sigma, (T)lam, (T)rho, (T)(1.0 - rho), relax == 0, h_kind == 1, w, z, z_out, st);
}

// dense tap window (index t + R) of one axis from (offset, coefficient) lists; returns the radius or -1
inline int tap_window(int nt, const int32_t* off, const double* coef, double (&k)[2 * kMaxR + 1]) {
  for (double& v : k) v = 0.0;
  int R = 0;
  for (int q = 0; q < nt; ++q) R = abs(off[q]) > R ? abs(off[q]) : R;
  if (R > kMaxR) return -1;
  for (int q = 0; q < nt; ++q) k[off[q] + kMaxR] += coef[q];
  return R;
}

// Measurement hook (PXA_TUNE_PDS_EVENTS > 0, bench.py's c3 record): HIP events recorded on the launch stream
// before kernel A and after kernels A, B and C of every step, so that the per-kernel times of the timed
// steps are read afterwards (pxa_pds_kernel_ms) without synchronising inside the timed region.
constexpr int kPdsEventSteps = 64;
struct PdsEvents {
  hipEvent_t ev[kPdsEventSteps][4];
  int created = 0;  // steps whose events exist
  int used = 0;     // steps recorded since the last read
};
static PdsEvents g_pds_ev;

static void pds_event(int k, hipStream_t st) {
  PdsEvents& E = g_pds_ev;
  if (E.used >= kPdsEventSteps) return;
  if (E.used == E.created) {
    for (int j = 0; j < 4; ++j) (void)hipEventCreate(&E.ev[E.created][j]);
    ++E.created;
  }
  (void)hipEventRecord(E.ev[E.used][k], st);
  if (k == 3) ++E.used;
}

// Validated geometry, taps and scalars shared by the three-launch and the look-ahead step.
template <typename T>
struct PdsSetup {
  PdsGeom<T> g;
  double kw[3][2 * kMaxR + 1];
  int R0, R;  // axis-0 radius (0: axis 0 not blurred), in-plane radius
  bool id0;
  T tau, sigma, rho, lam, pw, omr;
  int64_t M;
  int prox;
  bool iso;
};

template <typename T>
int pds_setup(const int64_t* geom, const int32_t* ntaps, const int32_t* offs, const double* coefs, const double* diff,
              const double* scal, int prox, int h_kind, PdsSetup<T>& S) {
  PXA_CHECK_ARG(geom && ntaps && offs && coefs && diff && scal);
  const int64_t stack = geom[0], y_images = geom[1], n0 = geom[2], n1 = geom[3], n2 = geom[4], D = geom[5];
  PXA_CHECK_ARG(stack >= 1 && y_images >= 1 && stack % y_images == 0);
  PXA_CHECK_ARG(n0 >= 1 && n1 >= 1 && n2 >= 1 && n0 <= 0x7fffffff && n1 <= 0x7fffffff && n2 <= 0x7fffffff);
  PXA_CHECK_ARG(D == 2 || D == 3);
  PXA_CHECK_ARG(stack <= 65535 && n0 * n1 * n2 <= ((int64_t)1 << 40));
  PXA_CHECK_ARG(prox >= 0 && prox <= 2 && (h_kind == 0 || h_kind == 1));
  for (int a = 0; a < 3; ++a) PXA_CHECK_ARG(ntaps[a] >= 1 && ntaps[a] <= 2 * kMaxR + 1);
  int Ra[3];
  for (int a = 0; a < 3; ++a) {
    Ra[a] = tap_window(ntaps[a], offs + a * (2 * kMaxR + 1), coefs + a * (2 * kMaxR + 1), S.kw[a]);
    if (Ra[a] < 0) return PXA_ERR_UNSUPPORTED;
  }
  // axis 0 is the identity iff its window is exactly [1] at offset 0
  S.id0 = Ra[0] == 0 && S.kw[0][kMaxR] == 1.0;
  S.R0 = S.id0 ? 0 : (Ra[0] > 0 ? Ra[0] : 1);
  S.R = Ra[1] > Ra[2] ? Ra[1] : Ra[2];
  if (S.R < 1) S.R = 1;
  PdsGeom<T>& g = S.g;
  g.stack = stack;
  g.y_images = y_images;
  g.n0 = (int)n0;
  g.n1 = (int)n1;
  g.n2 = (int)n2;
  g.D = (int)D;
  for (int a = 0; a < 3; ++a) {
    g.c0[a] = (T)diff[a];
    g.c1[a] = (T)diff[3 + a];
  }
  S.tau = (T)scal[0];
  S.sigma = (T)scal[1];
  S.rho = (T)scal[2];
  S.lam = (T)scal[3];
  S.pw = (T)scal[4];
  S.omr = (T)(1.0 - scal[2]);
  S.M = n1 * n2;
  S.prox = prox;
  S.iso = h_kind == 1;
  return PXA_OK;
}

// axis-0 march parameters (kernels A and D); resolves nseg (< 1: auto)
template <typename T>
PdsA<T> make_a(const PdsSetup<T>& S, int& nseg) {
  PdsA<T> pa;
  pa.g = S.g;
  for (int t = 0; t < 2 * kMaxR0 + 1; ++t) pa.k0[t] = T(0);
  for (int t = -S.R0; t <= S.R0; ++t) pa.k0[t + S.R0] = (T)S.kw[0][t + kMaxR];
  pa.tau = S.tau;
  pa.pw = S.pw;
  pa.prox = S.prox;
  const int64_t n0 = S.g.n0;
  if (nseg < 1) {
    // auto: about 4096 workgroups in flight, segments >= 4 rings deep (halo recompute <= 1/2)
    const int64_t blocks = S.g.stack * ((S.M + 2 * kAThreads - 1) / (2 * kAThreads));
    const int64_t want = (4096 + blocks - 1) / blocks;
    const int64_t cap = S.R0 > 0 ? n0 / (4 * (2 * S.R0 + 1)) : n0;
    nseg = (int)(want < cap ? want : cap);
    if (nseg < 1) nseg = 1;
  }
  if (nseg > n0) nseg = (int)n0;
  pa.seg = (int)((n0 + nseg - 1) / nseg);
  nseg = (int)((n0 + pa.seg - 1) / pa.seg);
  return pa;
}

// kernel B: mode 0 PD3O, 1 Condat-Vu (K^T z from z), 2 Condat-Vu (K^T z given in `z`)
template <typename T>
int stage_b(const PdsSetup<T>& S, int mode, const void* q_src, const void* xin, const void* u, const void* z,
            const void* hty, void* w, void* out, hipStream_t st) {
  constexpr int V = kVecN<T>;
  const int R = S.R;
  PdsB<T> pb;
  pb.g = S.g;
  pb.tiles1 = (int)((S.g.n1 + TY - 1) / TY);
  pb.tiles2 = (int)((S.g.n2 + TX - 1) / TX);
  const int64_t ntiles = S.g.stack * S.g.n0 * pb.tiles1 * pb.tiles2;
  PXA_CHECK_ARG(ntiles <= 0x7fffffff);
  pb.ntiles = (unsigned)ntiles;
  for (int j = 0; j < 2 * kMaxR + 1; ++j) pb.k1[j] = pb.k2[j] = T(0);
  for (int t = -R; t <= R; ++t) {
    pb.k1[t + R] = (T)S.kw[1][t + kMaxR];
    pb.k2[t + R] = (T)S.kw[2][t + kMaxR];
  }
  for (int j = 0; j < kMaxG; ++j) pb.g1[j] = pb.g2[j] = T(0);
  for (int d = -2 * R; d <= 2 * R; ++d) {
    double s1 = 0.0, s2 = 0.0;
    for (int t = -R; t <= R; ++t) {
      if (t + d < -R || t + d > R) continue;
      s1 += S.kw[1][t + kMaxR] * S.kw[1][t + d + kMaxR];
      s2 += S.kw[2][t + kMaxR] * S.kw[2][t + d + kMaxR];
    }
    pb.g1[d + 2 * R] = (T)s1;
    pb.g2[d + 2 * R] = (T)s2;
  }
  pb.tau = S.tau;
  pb.rho = S.rho;
  pb.omr = S.omr;
  pb.pw = S.pw;
  pb.prox = S.prox;
  pb.vec_ok = (S.g.n2 % V == 0) && aligned16(q_src) && aligned16(xin) && aligned16(hty) && aligned16(w) &&
              aligned16(out) && aligned16(z) && (mode != 0 || aligned16(u));
  PdsPtrs P{q_src, xin, u, z, hty, w, out};
  return run_b(pb, mode, R, P, st);
}

template <typename T>
int pds_entry(int algo, const int64_t* geom, const int32_t* ntaps, const int32_t* offs, const double* coefs,
              const double* diff, const double* scal, int prox, int h_kind, const void* x, const void* u,
              const void* z, const void* hty, void* x_out, void* u_out, void* z_out, void* work_q, void* work_w,
              int nseg, hipStream_t st) {
  PXA_CHECK_ARG(algo == 0 || algo == 1);
  PdsSetup<T> S;
  if (const int e = pds_setup<T>(geom, ntaps, offs, coefs, diff, scal, prox, h_kind, S)) return e;
  const bool pd3o = algo == 0;
  PXA_CHECK_ARG(z && hty && z_out && work_w && x_out && (pd3o ? (u && u_out) : (x != nullptr)));
  PXA_CHECK_ARG(pd3o || x_out != x);  // kernel B reads x windows (halos) while writing x_out
  if (!S.id0) PXA_CHECK_ARG(work_q != nullptr);
  const PdsGeom<T>& g = S.g;
  const int64_t M = S.M;

  const bool evs = tuning(PXA_TUNE_PDS_EVENTS) > 0;
  if (evs) pds_event(0, st);
  // ---- kernel A
  const void* q_src = pd3o ? (const void*)x_out : x;  // kernel B's input plane stack
  if (pd3o || !S.id0) {
    const PdsA<T> pa = make_a(S, nseg);
    const void* src = pd3o ? u : x;
    const bool np2 = (g.n2 % 2 == 0) && ((uintptr_t)src % (2 * sizeof(T)) == 0) &&
                     ((uintptr_t)z % (2 * sizeof(T)) == 0) && ((uintptr_t)x_out % (2 * sizeof(T)) == 0) &&
                     (S.id0 || (uintptr_t)work_q % (2 * sizeof(T)) == 0);
    void* q = S.id0 ? x_out : work_q;  // R0 == 0 never writes q
    const int e = run_a(pa, pd3o, S.R0, np2 ? 2 : 1, M, nseg, src, z, x_out, q, st);
    if (e) return e;
    if (!S.id0) q_src = work_q;
  }
  if (evs) pds_event(1, st);

  // ---- kernel B
  {
    const int e = stage_b(S, pd3o ? 0 : 1, q_src, pd3o ? (const void*)x_out : x, u, z, hty, work_w,
                          pd3o ? u_out : x_out, st);
    if (e) return e;
  }
  if (evs) pds_event(2, st);

  // ---- kernel C
  if (const int e = run_c<T>(g, S.sigma, S.lam, S.rho, S.omr, pd3o, S.iso, work_w, z, z_out, st)) return e;
  if (evs) pds_event(3, st);
  return PXA_OK;
}

// Look-ahead step (pds_march.hpp): [priming march] + kernel B + kernel D.  PD3O: x (current x; written by
// the priming march unless primed), u -> u_out, z -> z_out, x_out = x of the next iteration.  Condat-Vu:
// x -> x_out, z -> z_out, work_kt = K^T z (written by the priming march unless primed, then rewritten for
// the next iteration).  work_q = G0 v (same priming rule; rewritten by kernel D).
template <typename T>
int pds_la_entry(int algo, const int64_t* geom, const int32_t* ntaps, const int32_t* offs, const double* coefs,
                 const double* diff, const double* scal, int prox, int h_kind, int primed, void* x, const void* u,
                 const void* z, const void* hty, void* x_out, void* u_out, void* z_out, void* work_q, void* work_kt,
                 void* work_w, int nseg, hipStream_t st) {
  PXA_CHECK_ARG(algo == 0 || algo == 1);
  PdsSetup<T> S;
  if (const int e = pds_setup<T>(geom, ntaps, offs, coefs, diff, scal, prox, h_kind, S)) return e;
  const bool pd3o = algo == 0;
  PXA_CHECK_ARG(x && z && hty && z_out && work_w && x_out && x_out != x && z_out != z);
  PXA_CHECK_ARG(pd3o ? (u && u_out) : (work_kt != nullptr));
  if (!S.id0) PXA_CHECK_ARG(work_q != nullptr);
  const PdsGeom<T>& g = S.g;
  const int64_t M = S.M;
  PdsD<T> pd;
  pd.a = make_a(S, nseg);
  pd.sigma = S.sigma;
  pd.lam = S.lam;
  pd.rho = S.rho;
  pd.omr = S.omr;
  // kernel D's per-thread pairs: even rows and 8-byte aligned streams
  auto a2 = [](const void* p) { return p == nullptr || (uintptr_t)p % (2 * sizeof(T)) == 0; };
  const bool np2 = (g.n2 % 2 == 0) && a2(x) && a2(u) && a2(z) && a2(x_out) && a2(u_out) && a2(z_out) &&
                   a2(work_q) && a2(work_kt) && a2(work_w);
  const int np = np2 ? 2 : 1;
  // q is written only when axis 0 is blurred; kernel B then reads it, else v itself
  void* q = S.id0 ? work_w : work_q;

  const bool evs = tuning(PXA_TUNE_PDS_EVENTS) > 0;
  if (evs) pds_event(0, st);
  if (!primed) {  // the march of this iteration: v from (u or x, z) without a dual update
    const int e = run_d(pd, pd3o, S.iso, false, S.R0, np, M, nseg, work_w, z, pd3o ? u : x, z_out,
                        pd3o ? x : work_kt, q, st);
    if (e) return e;
  }
  if (evs) pds_event(1, st);
  {
    const void* q_src = S.id0 ? (const void*)x : work_q;
    const int e = pd3o ? stage_b(S, 0, q_src, x, u, z, hty, work_w, u_out, st)
                       : stage_b(S, 2, q_src, x, nullptr, work_kt, hty, work_w, x_out, st);
    if (e) return e;
  }
  if (evs) pds_event(2, st);
  {
    // dual update of this iteration + the next iteration's march
    const int e = run_d(pd, pd3o, S.iso, true, S.R0, np, M, nseg, work_w, z, pd3o ? (const void*)u_out : x_out,
                        z_out, pd3o ? x_out : work_kt, q, st);
    if (e) return e;
  }
  if (evs) pds_event(3, st);
  return PXA_OK;
}

}  // namespace pds
}  // namespace pxa

using namespace pxa::pds;
using namespace pxa;

extern "C" {

int pxa_pds_kernel_ms(double* ms_abc, int reset) {
  PdsEvents& E = g_pds_ev;
  if (!ms_abc) return PXA_ERR_ARG;
  ms_abc[0] = ms_abc[1] = ms_abc[2] = 0.0;
  const int n = E.used;
  if (n > 0 && hipEventSynchronize(E.ev[n - 1][3]) != hipSuccess) return PXA_ERR_UNSUPPORTED;
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, E.ev[i][k], E.ev[i][k + 1]) != hipSuccess) return PXA_ERR_UNSUPPORTED;
      ms_abc[k] += ms;
    }
  if (reset) E.used = 0;
  return n;
}

int pxa_pds_step(int dtype, int algo, const int64_t* geom, const int32_t* ntaps, const int32_t* offs,
                 const double* coefs, const double* diff, const double* scal, int prox, int h_kind, const void* x,
                 const void* u, const void* z, const void* hty, void* x_out, void* u_out, void* z_out, void* work_q,
                 void* work_w, int nseg, void* stream) {
  PXA_DISPATCH(dtype, T,
               return pds_entry<T>(algo, geom, ntaps, offs, coefs, diff, scal, prox, h_kind, x, u, z, hty, x_out, u_out,
                                   z_out, work_q, work_w, nseg, as_stream(stream)));
}

int pxa_tv_dual_update(int dtype, int relax, const int64_t* geom, const double* diff, double sigma, double lam,
                       double rho, int h_kind, const void* w, const void* z, void* z_out, void* stream) {
  PXA_DISPATCH(dtype, T,
               return dual_entry<T>(relax, geom, diff, sigma, lam, rho, h_kind, w, z, z_out, as_stream(stream)));
}

int pxa_pds_step_la(int dtype, int algo, const int64_t* geom, const int32_t* ntaps, const int32_t* offs,
                    const double* coefs, const double* diff, const double* scal, int prox, int h_kind, int primed,
                    void* x, const void* u, const void* z, const void* hty, void* x_out, void* u_out, void* z_out,
                    void* work_q, void* work_kt, void* work_w, int nseg, void* stream) {
  PXA_DISPATCH(dtype, T,
               return pds_la_entry<T>(algo, geom, ntaps, offs, coefs, diff, scal, prox, h_kind, primed, x, u, z, hty,
                                      x_out, u_out, z_out, work_q, work_kt, work_w, nseg, as_stream(stream)));
}

}  // extern "C"
