// Gradient = vstack of 2-tap finite-difference Stencils, evaluated in one pass (apply and adjoint).
//
// apply  : reads x once (+ one neighbour per direction from L1/L2), writes ndir fields;
// adjoint: reads ndir fields (+ one neighbour each), writes one field.
// Both stream whole rows: the per-element index arithmetic of a flat grid-stride loop (64-bit
// divisions per direction) made the first version ALU-bound at 1.7 TB/s on 1024^3.
// Zero (constant-mode) boundary, exactly Trim o S o Pad of the reference per direction.
#include "common.hpp"

namespace pxa {
namespace {

template <typename T>
struct Dirs {
  int n;
  int64_t st[PXA_MAX_DIM];  // stride of the differentiated axis, per direction
  int64_t len[PXA_MAX_DIM]; // length of that axis
  int64_t ax_st[PXA_MAX_DIM];
  int o0[PXA_MAX_DIM], o1[PXA_MAX_DIM];
  T c0[PXA_MAX_DIM], c1[PXA_MAX_DIM];
  bool one0[PXA_MAX_DIM], one1[PXA_MAX_DIM];  // tap == 1 exactly: no multiply (codegen rule)
};

template <typename T>
__device__ inline T tap(T c, bool one, T v) {
  return one ? v : c * v;
}

// Row-structured kernels: a workgroup item is one (row, column block) of the volume, a thread owns V
// consecutive elements of the last axis.  Every coordinate except the last is uniform per item
// (scalar arithmetic); off-last-axis neighbours are whole-vector loads at +-stride, last-axis
// neighbours are per-element loads that hit the cache lines of the vector itself.
// n / d for 32-bit n by one multiply-high (Granlund-Montgomery, exact for every 32-bit n; built on the host)
struct U32Div {
  uint32_t d = 1, m = 1;
  int s = 0;
  void set(uint32_t dd) {
    d = dd;
    s = 0;
    while ((1ull << s) < dd) ++s;
    m = (uint32_t)(((1ull << 32) * ((1ull << s) - dd)) / dd + 1);
  }
  __device__ uint32_t div(uint32_t n) const {
    const uint32_t t = __umulhi(n, m);
    return (uint32_t)(((uint64_t)t + n) >> s);
  }
};

struct RowGeom {
  int64_t rows_per_vol;  // N / n_last
  int n_last;
  int cblocks;
  int64_t items;                  // stack * rows_per_vol * cblocks
  int last[PXA_MAX_DIM];          // direction d differentiates the last axis
  int64_t rstride[PXA_MAX_DIM];   // stride of the direction's axis in rows (non-last axes)
  // items < 2^31: the item -> (volume, row, column block, axis coordinate) divisions in 32 bits
  bool small;
  U32Div dcb, drpv, drst[PXA_MAX_DIM], dlen[PXA_MAX_DIM];
};

template <typename T, int V>
__device__ inline void ldv(const T* p, T (&v)[V]) {
  if constexpr (V == kVecN<T>)
    *reinterpret_cast<typename Vec4<T>::type*>(v) = *reinterpret_cast<const typename Vec4<T>::type*>(p);
  else
    v[0] = p[0];
}
template <typename T, int V>
__device__ inline void stv(T* p, const T (&v)[V]) {
  if constexpr (V == kVecN<T>)
    *reinterpret_cast<typename Vec4<T>::type*>(p) = *reinterpret_cast<const typename Vec4<T>::type*>(v);
  else
    p[0] = v[0];
}

// values of x at i0 + e + o (e < V) along direction d, zero outside the axis (constant mode)
template <typename T, int V>
__device__ inline void neighbour(const T* __restrict__ xs, int64_t i0, int c, int64_t rin, int d, int o,
                                 const Dirs<T>& dd, const RowGeom& g, T (&v)[V]) {
  if (g.last[d]) {
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const int cc = c + e + o;
      v[e] = (cc >= 0 && cc < g.n_last) ? xs[i0 + e + o] : T(0);
    }
  } else {
    const int64_t ca = (rin / g.rstride[d]) % dd.len[d] + o;
    if (ca >= 0 && ca < dd.len[d]) {
      ldv<T, V>(xs + i0 + (int64_t)o * dd.st[d], v);
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) v[e] = T(0);
    }
  }
}

// non-temporal store: the outputs are written once and never re-read here, so they should not evict the
// input rows whose neighbours other workgroups read from L2
template <typename T, int V>
__device__ inline void stv_nt(T* p, const T (&v)[V]) {
  if constexpr (V == 1) {
    __builtin_nontemporal_store(v[0], p);
  } else {
    typedef T vt __attribute__((ext_vector_type(V)));
    vt r;
#pragma unroll
    for (int i = 0; i < V; ++i) r[i] = v[i];
    __builtin_nontemporal_store(r, reinterpret_cast<vt*>(p));
  }
}

__device__ inline unsigned band_xcd(unsigned bid, unsigned nb) {  // XCD g = bid % 8 takes a contiguous band
  const unsigned q8 = nb >> 3, r8 = nb & 7u, g8 = bid & 7u;
  return g8 * q8 + (g8 < r8 ? g8 : r8) + (bid >> 3);
}

// values of x at i0 + e + o (e < V) along direction d, given the centre vector xc = x[i0 .. i0 + V) and the
// item's coordinate ca along the direction's axis (non-last axes): |o| <= 1 on the last axis reuses xc and
// loads one scalar, o == 0 is xc itself, other axes one vector load
template <typename T, int V>
__device__ inline void neighbour_c(const T* __restrict__ xs, int64_t i0, int c, int64_t ca, int d, int o,
                                   const Dirs<T>& dd, const RowGeom& g, const T (&xc)[V], T (&v)[V]) {
  if (o == 0) {
#pragma unroll
    for (int e = 0; e < V; ++e) v[e] = xc[e];
  } else if (g.last[d]) {
    if (o == 1) {
#pragma unroll
      for (int e = 0; e + 1 < V; ++e) v[e] = xc[e + 1];
      v[V - 1] = c + V < g.n_last ? xs[i0 + V] : T(0);
    } else if (o == -1) {
#pragma unroll
      for (int e = V - 1; e > 0; --e) v[e] = xc[e - 1];
      v[0] = c > 0 ? xs[i0 - 1] : T(0);
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const int cc = c + e + o;
        v[e] = (cc >= 0 && cc < g.n_last) ? xs[i0 + e + o] : T(0);
      }
    }
  } else {
    if (ca + o >= 0 && ca + o < dd.len[d]) {
      ldv<T, V>(xs + i0 + (int64_t)o * dd.st[d], v);
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) v[e] = T(0);
    }
  }
}

// Two items per iteration (their loads issued before either is computed), the centre vector of each field
// loaded once, the item's axis coordinates once per direction (the first version: 10 load instructions per
// item for a 2-D forward gradient against 3 here, 0.34 of HBM at 2048^2 and 1024^3)
template <typename T, int V, bool ADJ>
__global__ void __launch_bounds__(kBlock) grad_rows_kernel(int64_t N, Dirs<T> dd, RowGeom g, const T* __restrict__ in,
                                                           T* __restrict__ out) {
  constexpr int U = 2;
  // XCD-banded: the workgroups of one XCD take consecutive items, so row + 1 is read from the same L2
  for (int64_t base = band_xcd(blockIdx.x, gridDim.x); base < g.items; base += (int64_t)U * gridDim.x) {
    T res[U][ADJ ? 1 : PXA_MAX_DIM][V];
    int64_t s_[U], i0_[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t item = base + (int64_t)u * gridDim.x;
      int64_t rowg, s, rin;
      if (g.small) {
        const uint32_t it = (uint32_t)item, rg = g.dcb.div(it), vs = g.drpv.div(rg);
        rowg = rg;
        s = vs;
        rin = rg - vs * (uint32_t)g.rows_per_vol;
      } else {
        rowg = item / g.cblocks;
        s = rowg / g.rows_per_vol;
        rin = rowg - s * g.rows_per_vol;
      }
      const int cb = (int)(item - rowg * g.cblocks);
      const int c = (cb * kBlock + (int)threadIdx.x) * V;
      ok[u] = item < g.items && c < g.n_last;
      s_[u] = i0_[u] = 0;
      if (!ok[u]) continue;
      // coordinate of the item's row along direction d's axis (non-last axes)
      auto coord = [&](int d) -> int64_t {
        if (g.last[d]) return 0;
        if (g.small) {
          const uint32_t q = g.drst[d].div((uint32_t)rin);
          return q - g.dlen[d].div(q) * g.dlen[d].d;
        }
        return (rin / g.rstride[d]) % dd.len[d];
      };
      const int64_t i0 = rin * g.n_last + c;
      s_[u] = s;
      i0_[u] = i0;
      if constexpr (!ADJ) {
        const T* xs = in + s * N;
        T xc[V];
        ldv<T, V>(xs + i0, xc);
#pragma unroll
        for (int d = 0; d < PXA_MAX_DIM; ++d) {
          if (d < dd.n) {
            const int64_t ca = coord(d);
            T v0[V], v1[V];
            neighbour_c<T, V>(xs, i0, c, ca, d, dd.o0[d], dd, g, xc, v0);
            neighbour_c<T, V>(xs, i0, c, ca, d, dd.o1[d], dd, g, xc, v1);
#pragma unroll
            for (int e = 0; e < V; ++e)
              res[u][d][e] = tap(dd.c0[d], dd.one0[d], v0[e]) + tap(dd.c1[d], dd.one1[d], v1[e]);
          }
        }
      } else {
#pragma unroll
        for (int d = 0; d < PXA_MAX_DIM; ++d) {
          if (d < dd.n) {
            const T* zd = in + (s * dd.n + d) * N;
            const int64_t ca = coord(d);
            T zc[V], v0[V], v1[V];
            ldv<T, V>(zd + i0, zc);
            // flipped kernel: taps (-o1, c1) then (-o0, c0)
            neighbour_c<T, V>(zd, i0, c, ca, d, -dd.o1[d], dd, g, zc, v1);
            neighbour_c<T, V>(zd, i0, c, ca, d, -dd.o0[d], dd, g, zc, v0);
#pragma unroll
            for (int e = 0; e < V; ++e) {
              const T term = tap(dd.c1[d], dd.one1[d], v1[e]) + tap(dd.c0[d], dd.one0[d], v0[e]);
              res[u][0][e] = (d == 0) ? term : res[u][0][e] + term;
            }
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      if constexpr (!ADJ) {
#pragma unroll
        for (int d = 0; d < PXA_MAX_DIM; ++d)
          if (d < dd.n) stv_nt<T, V>(out + (s_[u] * dd.n + d) * N + i0_[u], res[u][d]);
      } else {
        stv_nt<T, V>(out + s_[u] * N + i0_[u], res[u][0]);
      }
    }
  }
}

// ---- axis-0 march (ndim >= 2, rows of the last axis in whole 16-B vectors)
// A thread owns V consecutive in-plane elements and walks the planes of its axis-0 segment: each plane of
// the input is loaded once and carried as the axis-0 neighbour of the next (the row kernel above re-read
// it, and its grid order put row + 1 on another XCD: 3 x the input bytes fetched at 1024^3); in-plane
// blocks are XCD-banded, so the neighbours along the middle axes come from the L2 of the same XCD, where
// the adjacent block marches in step.  Outputs are written non-temporal.
struct MarchGeom {
  int n0;              // planes (axis 0)
  int seg;             // planes per axis-0 segment (grid.y)
  int64_t M;           // elements per plane
  int n_last;
  int ax[PXA_MAX_DIM];           // direction d's axis
  int64_t mst[PXA_MAX_DIM];      // its stride (middle axes; the last axis: 1)
  int64_t mlen[PXA_MAX_DIM];     // its length
  int last[PXA_MAX_DIM];          // the direction differentiates the last axis
};

template <typename T, int V, bool ADJ, bool NT>
__global__ void __launch_bounds__(kBlock) grad_march_kernel(int64_t N, Dirs<T> dd, MarchGeom g,
                                                            const T* __restrict__ in, T* __restrict__ out) {
  auto put = [](T* p, const T (&v)[V]) {
    if constexpr (NT) stv_nt<T, V>(p, v);
    else stv<T, V>(p, v);
  };
  const int64_t j0 = ((int64_t)band_xcd(blockIdx.x, gridDim.x) * kBlock + threadIdx.x) * V;
  if (j0 >= g.M) return;
  const int64_t s = blockIdx.z;
  const int pb = blockIdx.y * g.seg;
  const int pe = pb + g.seg < g.n0 ? pb + g.seg : g.n0;
  const int c = (int)(j0 % g.n_last);  // column of the first element in its row
  int64_t cm[PXA_MAX_DIM];             // in-plane coordinate along each middle-axis direction
#pragma unroll
  for (int d = 0; d < PXA_MAX_DIM; ++d)
    cm[d] = (d < dd.n && g.ax[d] > 0 && !g.last[d]) ? (j0 / g.mst[d]) % g.mlen[d] : 0;
  auto zero = [](T (&v)[V]) {
#pragma unroll
    for (int e = 0; e < V; ++e) v[e] = T(0);
  };
  // value at offset o of direction d (not axis 0) from the plane row xs + off, centre vector xc
  auto side = [&](const T* __restrict__ xs, int64_t off, int d, int o, const T (&xc)[V], T (&v)[V]) {
    if (o == 0) {
#pragma unroll
      for (int e = 0; e < V; ++e) v[e] = xc[e];
    } else if (g.last[d]) {
      if (o == 1) {
#pragma unroll
        for (int e = 0; e + 1 < V; ++e) v[e] = xc[e + 1];
        v[V - 1] = c + V < g.n_last ? xs[off + V] : T(0);
      } else if (o == -1) {
#pragma unroll
        for (int e = V - 1; e > 0; --e) v[e] = xc[e - 1];
        v[0] = c > 0 ? xs[off - 1] : T(0);
      } else {
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const int cc = c + e + o;
          v[e] = (cc >= 0 && cc < g.n_last) ? xs[off + e + o] : T(0);
        }
      }
    } else if (cm[d] + o >= 0 && cm[d] + o < g.mlen[d]) {
      ldv<T, V>(xs + off + (int64_t)o * g.mst[d], v);
    } else {
      zero(v);
    }
  };
  // axis-0 window of one field: w[0] = plane p - 1, w[1] = p, w[2] = p + 1 (zero outside [0, n0))
  auto plane = [&](const T* __restrict__ f, int p, T (&v)[V]) {
    if (p >= 0 && p < g.n0) ldv<T, V>(f + (int64_t)p * g.M + j0, v);
    else zero(v);
  };
  auto shift = [&](T (&w)[3][V], const T* __restrict__ f, int p) {  // to plane p: load p + 1
#pragma unroll
    for (int e = 0; e < V; ++e) {
      w[0][e] = w[1][e];
      w[1][e] = w[2][e];
    }
    plane(f, p + 1, w[2]);
  };
  auto a0 = [&](const T (&w)[3][V], int o, T (&v)[V]) {  // axis-0 neighbour at offset o in {-1, 0, 1} (selects:
#pragma unroll                                              // a runtime index would put w in scratch memory)
    for (int e = 0; e < V; ++e) v[e] = o < 0 ? w[0][e] : (o == 0 ? w[1][e] : w[2][e]);
  };
  if constexpr (!ADJ) {
    const T* xs = in + s * N;
    T w[3][V];
    plane(xs, pb - 1, w[1]);
    plane(xs, pb, w[2]);
    for (int p = pb; p < pe; ++p) {
      shift(w, xs, p);
      const int64_t off = (int64_t)p * g.M + j0;
#pragma unroll
      for (int d = 0; d < PXA_MAX_DIM; ++d) {
        if (d < dd.n) {
          T v0[V], v1[V], r[V];
          if (g.ax[d] == 0) {
            a0(w, dd.o0[d], v0);
            a0(w, dd.o1[d], v1);
          } else {
            side(xs, off, d, dd.o0[d], w[1], v0);
            side(xs, off, d, dd.o1[d], w[1], v1);
          }
#pragma unroll
          for (int e = 0; e < V; ++e) r[e] = tap(dd.c0[d], dd.one0[d], v0[e]) + tap(dd.c1[d], dd.one1[d], v1[e]);
          put(out + (s * dd.n + d) * N + off, r);
        }
      }
    }
  } else {
    // the axis-0 direction's field keeps a window; the others are read at the plane
    int d0 = -1;
#pragma unroll
    for (int d = 0; d < PXA_MAX_DIM; ++d)
      if (d < dd.n && g.ax[d] == 0 && d0 < 0) d0 = d;
    T w[3][V];
    zero(w[0]);
    zero(w[1]);
    zero(w[2]);
    const T* z0 = d0 >= 0 ? in + (s * dd.n + d0) * N : in;
    if (d0 >= 0) {
      plane(z0, pb - 1, w[1]);
      plane(z0, pb, w[2]);
    }
    for (int p = pb; p < pe; ++p) {
      if (d0 >= 0) shift(w, z0, p);
      const int64_t off = (int64_t)p * g.M + j0;
      T acc[V];
#pragma unroll
      for (int d = 0; d < PXA_MAX_DIM; ++d) {
        if (d < dd.n) {
          const T* zd = in + (s * dd.n + d) * N;
          T v0[V], v1[V];
          // flipped kernel: taps (-o1, c1) then (-o0, c0)
          if (d == d0) {
            a0(w, -dd.o1[d], v1);
            a0(w, -dd.o0[d], v0);
          } else if (g.ax[d] == 0) {  // a second axis-0 direction: plain loads
            plane(zd, p - dd.o1[d], v1);
            plane(zd, p - dd.o0[d], v0);
          } else {
            T zc[V];
            ldv<T, V>(zd + off, zc);
            side(zd, off, d, -dd.o1[d], zc, v1);
            side(zd, off, d, -dd.o0[d], zc, v0);
          }
#pragma unroll
          for (int e = 0; e < V; ++e) {
            const T term = tap(dd.c1[d], dd.one1[d], v1[e]) + tap(dd.c0[d], dd.one0[d], v0[e]);
            acc[e] = (d == 0) ? term : acc[e] + term;
          }
        }
      }
      put(out + s * N + off, acc);
    }
  }
}

template <typename T, bool ADJ>
int launch_rows(int64_t stack, int ndim, const int64_t* shape, int64_t N, const Dirs<T>& dd, const int* dirs,
                const void* in, void* out, hipStream_t st) {
  RowGeom g;
  g.n_last = (int)shape[ndim - 1];
  g.rows_per_vol = N / g.n_last;
  int64_t row_st[PXA_MAX_DIM];
  {
    int64_t s = 1;
    for (int a = ndim - 2; a >= 0; --a) {
      row_st[a] = s;
      s *= shape[a];
    }
  }
  for (int d = 0; d < PXA_MAX_DIM; ++d) {
    const bool valid = d < dd.n;
    g.last[d] = valid && dirs[d] == ndim - 1;
    g.rstride[d] = (valid && !g.last[d]) ? row_st[dirs[d]] : 1;
  }
  constexpr int V = kVecN<T>;
  const bool vec = g.n_last % V == 0 && aligned16(in) && aligned16(out);
  const int nv = vec ? V : 1;
  g.cblocks = (int)((g.n_last + (int64_t)kBlock * nv - 1) / ((int64_t)kBlock * nv));
  g.items = stack * g.rows_per_vol * g.cblocks;
  g.small = g.items + 2 * (int64_t)kMaxGrid < ((int64_t)1 << 31);
  if (g.small) {
    g.dcb.set((uint32_t)g.cblocks);
    g.drpv.set((uint32_t)g.rows_per_vol);
    for (int d = 0; d < PXA_MAX_DIM; ++d) {
      g.drst[d].set((uint32_t)g.rstride[d]);
      g.dlen[d].set((uint32_t)dd.len[d]);
    }
  }
  const int grid = (int)(g.items < (int64_t)kMaxGrid ? g.items : (int64_t)kMaxGrid);
  if (vec)
    hipLaunchKernelGGL((grad_rows_kernel<T, V, ADJ>), dim3(grid), dim3(kBlock), 0, st, N, dd, g, (const T*)in, (T*)out);
  else
    hipLaunchKernelGGL((grad_rows_kernel<T, 1, ADJ>), dim3(grid), dim3(kBlock), 0, st, N, dd, g, (const T*)in, (T*)out);
  return last_launch_status();
}


template <typename T, bool ADJ>
bool launch_march(int64_t stack, int ndim, const int64_t* shape, int64_t N, const Dirs<T>& dd, const int* dirs,
                  const void* in, void* out, hipStream_t st, int* status) {
  // planes of at least 64 K elements (64 workgroups of 1024 fp32 per plane): a 2048^2 image marched over
  // two-row segments took 39.5 us against 16 us for the row kernel (one latency round per row)
  if (ndim < 2 || stack > 65535 || shape[0] > 0x7fffffff || N / shape[0] < 65536) return false;
  for (int d = 0; d < dd.n; ++d)
    if (dirs[d] == 0 && (dd.o0[d] < -1 || dd.o0[d] > 1 || dd.o1[d] < -1 || dd.o1[d] > 1)) return false;
  MarchGeom g;
  g.n0 = (int)shape[0];
  g.M = N / g.n0;
  g.n_last = (int)shape[ndim - 1];
  for (int d = 0; d < PXA_MAX_DIM; ++d) {
    const bool valid = d < dd.n;
    g.ax[d] = valid ? dirs[d] : 0;
    g.last[d] = valid && dirs[d] == ndim - 1;
    g.mst[d] = valid ? dd.st[d] : 1;
    g.mlen[d] = valid ? dd.len[d] : 1;
  }
  constexpr int V = kVecN<T>;
  const bool vec = g.n_last % V == 0 && aligned16(in) && aligned16(out);
  const int nv = vec ? V : 1;
  const int64_t blocks = (g.M + (int64_t)kBlock * nv - 1) / ((int64_t)kBlock * nv);
  if (blocks > 0x7fffffff) return false;
  int64_t nseg = (2048 + blocks - 1) / blocks;  // about 2048 workgroups in flight
  if (nseg > g.n0) nseg = g.n0;
  if (nseg < 1) nseg = 1;
  g.seg = (int)((g.n0 + nseg - 1) / nseg);
  nseg = (g.n0 + g.seg - 1) / g.seg;
  const dim3 grid((unsigned)blocks, (unsigned)nseg, (unsigned)stack);
  const bool nt = !(tuning(PXA_TUNE_GRAD_KERNEL) & 2);  // bit 1: plain stores (A/B)
  if (vec && nt)
    hipLaunchKernelGGL((grad_march_kernel<T, V, ADJ, true>), grid, dim3(kBlock), 0, st, N, dd, g, (const T*)in, (T*)out);
  else if (vec)
    hipLaunchKernelGGL((grad_march_kernel<T, V, ADJ, false>), grid, dim3(kBlock), 0, st, N, dd, g, (const T*)in, (T*)out);
  else
    hipLaunchKernelGGL((grad_march_kernel<T, 1, ADJ, true>), grid, dim3(kBlock), 0, st, N, dd, g, (const T*)in, (T*)out);
  *status = last_launch_status();
  return true;
}

template <typename T>
bool make_dirs(int ndim, const int64_t* shape, int ndir, const int* dirs, const int* off0, const double* coef0,
               const int* off1, const double* coef1, Dirs<T>& dd, int64_t& N) {
  if (ndim < 1 || ndim > PXA_MAX_DIM || ndir < 1 || ndir > PXA_MAX_DIM) return false;
  if (!shape || !dirs || !off0 || !off1 || !coef0 || !coef1) return false;
  int64_t st[PXA_MAX_DIM];
  int64_t s = 1;
  for (int i = ndim - 1; i >= 0; --i) {
    if (shape[i] < 1) return false;
    st[i] = s;
    s *= shape[i];
  }
  N = s;
  dd.n = ndir;
  for (int d = 0; d < PXA_MAX_DIM; ++d) {
    if (d < ndir) {
      int a = dirs[d];
      if (a < 0 || a >= ndim) return false;
      dd.st[d] = st[a];
      dd.len[d] = shape[a];
      dd.o0[d] = off0[d];
      dd.o1[d] = off1[d];
      dd.c0[d] = (T)coef0[d];
      dd.c1[d] = (T)coef1[d];
      dd.one0[d] = coef0[d] == 1.0;
      dd.one1[d] = coef1[d] == 1.0;
    } else {
      dd.st[d] = 1;
      dd.len[d] = 1;
      dd.o0[d] = dd.o1[d] = 0;
      dd.c0[d] = dd.c1[d] = T(0);
      dd.one0[d] = dd.one1[d] = false;
    }
  }
  return true;
}

}  // namespace
}  // namespace pxa

using namespace pxa;

extern "C" {

int pxa_gradient2(int dtype, int64_t stack, int ndim, const int64_t* shape, int ndir, const int* dirs,
                  const int* off0, const double* coef0, const int* off1, const double* coef1, const void* x, void* g,
                  void* stream) {
  PXA_CHECK_ARG(stack >= 0);
  PXA_DISPATCH(dtype, T, {
    Dirs<T> dd;
    int64_t N;
    PXA_CHECK_ARG(make_dirs<T>(ndim, shape, ndir, dirs, off0, coef0, off1, coef1, dd, N));
    if (stack == 0) return PXA_OK;
    PXA_CHECK_ARG(x != nullptr && g != nullptr);
    PXA_CHECK_ARG(shape[ndim - 1] <= 0x7fffffff);
    int status = PXA_OK;
    if ((tuning(PXA_TUNE_GRAD_KERNEL) & 1) == 0 &&
        launch_march<T, false>(stack, ndim, shape, N, dd, dirs, x, g, as_stream(stream), &status))
      return status;
    return launch_rows<T, false>(stack, ndim, shape, N, dd, dirs, x, g, as_stream(stream));
  });
}

int pxa_gradient2_adjoint(int dtype, int64_t stack, int ndim, const int64_t* shape, int ndir, const int* dirs,
                          const int* off0, const double* coef0, const int* off1, const double* coef1, const void* z,
                          void* x, void* stream) {
  PXA_CHECK_ARG(stack >= 0);
  PXA_DISPATCH(dtype, T, {
    Dirs<T> dd;
    int64_t N;
    PXA_CHECK_ARG(make_dirs<T>(ndim, shape, ndir, dirs, off0, coef0, off1, coef1, dd, N));
    if (stack == 0) return PXA_OK;
    PXA_CHECK_ARG(z != nullptr && x != nullptr);
    PXA_CHECK_ARG(shape[ndim - 1] <= 0x7fffffff);
    int status = PXA_OK;
    if ((tuning(PXA_TUNE_GRAD_KERNEL) & 1) == 0 &&
        launch_march<T, true>(stack, ndim, shape, N, dd, dirs, z, x, as_stream(stream), &status))
      return status;
    return launch_rows<T, true>(stack, ndim, shape, N, dd, dirs, z, x, as_stream(stream));
  });
}

}  // extern "C"
