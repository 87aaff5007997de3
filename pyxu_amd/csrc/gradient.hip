// Gradient = vstack of 2-tap finite-difference Stencils, evaluated in one pass (apply and adjoint).
//
// apply  : reads x once (+ one neighbour per direction from L1/L2), writes ndir fields;
// adjoint: reads ndir fields (+ one neighbour each), writes one field.
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

template <typename T>
__global__ void __launch_bounds__(kBlock) grad_kernel(int64_t stack, int64_t N, Dirs<T> dd, const T* __restrict__ x,
                                                      T* __restrict__ g) {
  const int64_t total = stack * N;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    int64_t s = t / N, i = t - s * N;
    const T* xs = x + s * N;
    T* gs = g + s * dd.n * N;
#pragma unroll
    for (int d = 0; d < PXA_MAX_DIM; ++d) {
      if (d < dd.n) {
        int64_t c = (i / dd.st[d]) % dd.len[d];
        int64_t c0 = c + dd.o0[d], c1 = c + dd.o1[d];
        T v0 = (c0 >= 0 && c0 < dd.len[d]) ? xs[i + dd.o0[d] * dd.st[d]] : T(0);
        T v1 = (c1 >= 0 && c1 < dd.len[d]) ? xs[i + dd.o1[d] * dd.st[d]] : T(0);
        gs[d * N + i] = tap(dd.c0[d], dd.one0[d], v0) + tap(dd.c1[d], dd.one1[d], v1);
      }
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) grad_adj_kernel(int64_t stack, int64_t N, Dirs<T> dd,
                                                          const T* __restrict__ z, T* __restrict__ x) {
  const int64_t total = stack * N;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    int64_t s = t / N, i = t - s * N;
    const T* zs = z + s * dd.n * N;
    T acc = T(0);
#pragma unroll
    for (int d = 0; d < PXA_MAX_DIM; ++d) {
      if (d < dd.n) {
        const T* zd = zs + d * N;
        int64_t c = (i / dd.st[d]) % dd.len[d];
        // flipped kernel: taps (-o1, c1) then (-o0, c0)
        int64_t a1 = c - dd.o1[d], a0 = c - dd.o0[d];
        T v1 = (a1 >= 0 && a1 < dd.len[d]) ? zd[i - dd.o1[d] * dd.st[d]] : T(0);
        T v0 = (a0 >= 0 && a0 < dd.len[d]) ? zd[i - dd.o0[d] * dd.st[d]] : T(0);
        T term = tap(dd.c1[d], dd.one1[d], v1) + tap(dd.c0[d], dd.one0[d], v0);
        acc = (d == 0) ? term : acc + term;
      }
    }
    x[t] = acc;
  }
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
    hipLaunchKernelGGL((grad_kernel<T>), dim3(grid_for(stack * N)), dim3(kBlock), 0, as_stream(stream), stack, N, dd,
                       (const T*)x, (T*)g);
    return last_launch_status();
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
    hipLaunchKernelGGL((grad_adj_kernel<T>), dim3(grid_for(stack * N)), dim3(kBlock), 0, as_stream(stream), stack, N,
                       dd, (const T*)z, (T*)x);
    return last_launch_status();
  });
}

}  // extern "C"
