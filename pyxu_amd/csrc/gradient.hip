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
struct RowGeom {
  int64_t rows_per_vol;  // N / n_last
  int n_last;
  int cblocks;
  int64_t items;                  // stack * rows_per_vol * cblocks
  int last[PXA_MAX_DIM];          // direction d differentiates the last axis
  int64_t rstride[PXA_MAX_DIM];   // stride of the direction's axis in rows (non-last axes)
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

template <typename T, int V, bool ADJ>
__global__ void __launch_bounds__(kBlock) grad_rows_kernel(int64_t N, Dirs<T> dd, RowGeom g, const T* __restrict__ in,
                                                           T* __restrict__ out) {
  for (int64_t item = blockIdx.x; item < g.items; item += gridDim.x) {
    const int64_t rowg = item / g.cblocks;
    const int cb = (int)(item - rowg * g.cblocks);
    const int c = (cb * kBlock + (int)threadIdx.x) * V;
    if (c >= g.n_last) continue;
    const int64_t s = rowg / g.rows_per_vol, rin = rowg - s * g.rows_per_vol;
    const int64_t i0 = rin * g.n_last + c;
    if constexpr (!ADJ) {
      const T* xs = in + s * N;
#pragma unroll
      for (int d = 0; d < PXA_MAX_DIM; ++d) {
        if (d < dd.n) {
          T v0[V], v1[V], r[V];
          neighbour<T, V>(xs, i0, c, rin, d, dd.o0[d], dd, g, v0);
          neighbour<T, V>(xs, i0, c, rin, d, dd.o1[d], dd, g, v1);
#pragma unroll
          for (int e = 0; e < V; ++e) r[e] = tap(dd.c0[d], dd.one0[d], v0[e]) + tap(dd.c1[d], dd.one1[d], v1[e]);
          stv<T, V>(out + (s * dd.n + d) * N + i0, r);
        }
      }
    } else {
      T acc[V];
#pragma unroll
      for (int d = 0; d < PXA_MAX_DIM; ++d) {
        if (d < dd.n) {
          const T* zd = in + (s * dd.n + d) * N;
          T v0[V], v1[V];
          // flipped kernel: taps (-o1, c1) then (-o0, c0)
          neighbour<T, V>(zd, i0, c, rin, d, -dd.o1[d], dd, g, v1);
          neighbour<T, V>(zd, i0, c, rin, d, -dd.o0[d], dd, g, v0);
#pragma unroll
          for (int e = 0; e < V; ++e) {
            const T term = tap(dd.c1[d], dd.one1[d], v1[e]) + tap(dd.c0[d], dd.one0[d], v0[e]);
            acc[e] = (d == 0) ? term : acc[e] + term;
          }
        }
      }
      stv<T, V>(out + s * N + i0, acc);
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
  const int grid = (int)(g.items < (int64_t)kMaxGrid ? g.items : (int64_t)kMaxGrid);
  if (vec)
    hipLaunchKernelGGL((grad_rows_kernel<T, V, ADJ>), dim3(grid), dim3(kBlock), 0, st, N, dd, g, (const T*)in, (T*)out);
  else
    hipLaunchKernelGGL((grad_rows_kernel<T, 1, ADJ>), dim3(grid), dim3(kBlock), 0, st, N, dd, g, (const T*)in, (T*)out);
  return last_launch_status();
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
    return launch_rows<T, true>(stack, ndim, shape, N, dd, dirs, z, x, as_stream(stream));
  });
}

}  // extern "C"
