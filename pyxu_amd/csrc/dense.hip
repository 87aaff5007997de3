// Dense LinOp (_ExplicitLinOp): Y = X A^T (apply) and Y = X A (adjoint), A row-major (M x N).
//
// HBM-bound for small stacks B (intensity 0.5*B flop/B): stream A exactly once
// with 16 B/lane loads and keep B running sums per lane in registers (B processed in register
// chunks of kBC).  apply: one wavefront per row of A; adjoint: workgroups own (row-chunk x
// column-tile) panels, write partial sums, a second pass adds the chunks in a fixed order.
#include "common.hpp"

namespace pxa {
namespace {

constexpr int kBC = 8;  // stacked right-hand sides per register chunk

// ------------------------------------------------------------------ apply: Y[b, m] = <A[m,:], X[b,:]>
template <typename T>
__global__ void __launch_bounds__(kBlock) gemv_rows_kernel(int64_t M, int64_t N, int64_t B, int64_t b0, int nb,
                                                           const T* __restrict__ A, const T* __restrict__ X,
                                                           T* __restrict__ Y, bool vec) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  constexpr int V = kVecN<T>;
  using VT = typename Vec4<T>::type;
  for (int64_t m = wave; m < M; m += nwaves) {
    const T* a = A + m * N;
    double acc[kBC];
#pragma unroll
    for (int j = 0; j < kBC; ++j) acc[j] = 0.0;
    if (vec) {
      for (int64_t k = (int64_t)lane * V; k < N; k += 64 * V) {
        T av[V];
        *reinterpret_cast<VT*>(av) = *reinterpret_cast<const VT*>(a + k);
#pragma unroll
        for (int j = 0; j < kBC; ++j) {
          if (j < nb) {
            T xv[V];
            *reinterpret_cast<VT*>(xv) = *reinterpret_cast<const VT*>(X + (b0 + j) * N + k);
            T part = T(0);
#pragma unroll
            for (int v = 0; v < V; ++v) part += av[v] * xv[v];
            acc[j] += (double)part;
          }
        }
      }
    } else {
      for (int64_t k = lane; k < N; k += 64) {
        T av = a[k];
#pragma unroll
        for (int j = 0; j < kBC; ++j)
          if (j < nb) acc[j] += (double)(av * X[(b0 + j) * N + k]);
      }
    }
#pragma unroll
    for (int j = 0; j < kBC; ++j) {
      double v = acc[j];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
      if (lane == 0 && j < nb) Y[(b0 + j) * M + m] = (T)v;
    }
  }
}

// ------------------------------------------------------------------ adjoint: Y[b, n] = sum_m A[m,n] X[b,m]
constexpr int kRowChunk = 128;

template <typename T>
__global__ void __launch_bounds__(kBlock) gemv_cols_partial_kernel(int64_t M, int64_t N, int64_t B, int64_t b0, int nb,
                                                                   const T* __restrict__ A, const T* __restrict__ X,
                                                                   T* __restrict__ part, bool vec) {
  constexpr int V = kVecN<T>;
  using VT = typename Vec4<T>::type;
  const int64_t chunk = blockIdx.y;
  const int64_t m_lo = chunk * kRowChunk;
  const int64_t m_hi = m_lo + kRowChunk < M ? m_lo + kRowChunk : M;
  const int64_t n0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * V;
  if (n0 >= N) return;
  T acc[kBC][V];
#pragma unroll
  for (int j = 0; j < kBC; ++j)
#pragma unroll
    for (int v = 0; v < V; ++v) acc[j][v] = T(0);
  for (int64_t m = m_lo; m < m_hi; ++m) {
    T av[V];
    if (vec && n0 + V <= N) {
      *reinterpret_cast<VT*>(av) = *reinterpret_cast<const VT*>(A + m * N + n0);
    } else {
#pragma unroll
      for (int v = 0; v < V; ++v) av[v] = (n0 + v < N) ? A[m * N + n0 + v] : T(0);
    }
#pragma unroll
    for (int j = 0; j < kBC; ++j) {
      if (j < nb) {
        T xm = X[(b0 + j) * M + m];
#pragma unroll
        for (int v = 0; v < V; ++v) acc[j][v] += av[v] * xm;
      }
    }
  }
  // part layout: (chunks, kBC, N)
  T* p = part + chunk * kBC * N;
#pragma unroll
  for (int j = 0; j < kBC; ++j)
    if (j < nb)
#pragma unroll
      for (int v = 0; v < V; ++v)
        if (n0 + v < N) p[j * N + n0 + v] = acc[j][v];
}

template <typename T>
__global__ void __launch_bounds__(kBlock) gemv_cols_final_kernel(int64_t M, int64_t N, int64_t b0, int nb,
                                                                 int64_t chunks, const T* __restrict__ part,
                                                                 T* __restrict__ Y) {
  const int64_t total = (int64_t)nb * N;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    int64_t j = t / N, n = t - j * N;
    double acc = 0.0;
    for (int64_t c = 0; c < chunks; ++c) acc += (double)part[(c * kBC + j) * N + n];
    Y[(b0 + j) * N + n] = (T)acc;
  }
}

}  // namespace
}  // namespace pxa

using namespace pxa;

extern "C" {

size_t pxa_dense_workspace_bytes(int dtype, int trans, int64_t M, int64_t N, int64_t B) {
  if (trans == 0) return 0;
  size_t es = dtype == PXA_F64 ? 8 : 4;
  int64_t chunks = (M + kRowChunk - 1) / kRowChunk;
  return (size_t)chunks * kBC * (size_t)N * es;
}

int pxa_dense_matmat(int dtype, int trans, int64_t M, int64_t N, int64_t B, const void* A, const void* X, void* Y,
                     void* work, void* stream) {
  PXA_CHECK_ARG(M >= 1 && N >= 1 && B >= 0);
  if (B == 0) return PXA_OK;
  PXA_CHECK_ARG(A != nullptr && X != nullptr && Y != nullptr);
  hipStream_t s = as_stream(stream);
  PXA_DISPATCH(dtype, T, {
    bool vec = aligned16(A) && aligned16(X) && (N % kVecN<T> == 0);
    if (trans == 0) {
      int64_t waves = M;
      int grid = grid_for(waves * 64);
      for (int64_t b0 = 0; b0 < B; b0 += kBC) {
        int nb = (int)(B - b0 < kBC ? B - b0 : kBC);
        hipLaunchKernelGGL((gemv_rows_kernel<T>), dim3(grid), dim3(kBlock), 0, s, M, N, B, b0, nb, (const T*)A,
                           (const T*)X, (T*)Y, vec);
        int e = last_launch_status();
        if (e) return e;
      }
      return PXA_OK;
    } else {
      PXA_CHECK_ARG(work != nullptr);
      int64_t chunks = (M + kRowChunk - 1) / kRowChunk;
      PXA_CHECK_ARG(chunks <= 65535);
      int64_t ntiles = (N + (int64_t)kBlock * kVecN<T> - 1) / ((int64_t)kBlock * kVecN<T>);
      bool vecA = aligned16(A) && (N % kVecN<T> == 0);
      for (int64_t b0 = 0; b0 < B; b0 += kBC) {
        int nb = (int)(B - b0 < kBC ? B - b0 : kBC);
        hipLaunchKernelGGL((gemv_cols_partial_kernel<T>), dim3((unsigned)ntiles, (unsigned)chunks), dim3(kBlock), 0, s,
                           M, N, B, b0, nb, (const T*)A, (const T*)X, (T*)work, vecA);
        int e = last_launch_status();
        if (e) return e;
        hipLaunchKernelGGL((gemv_cols_final_kernel<T>), dim3(grid_for((int64_t)nb * N)), dim3(kBlock), 0, s, M, N, b0,
                           nb, chunks, (const T*)work, (T*)Y);
        e = last_launch_status();
        if (e) return e;
      }
      return PXA_OK;
    }
  });
}

}  // extern "C"
