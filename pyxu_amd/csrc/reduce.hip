// Deterministic row reductions (RelError / AbsError norms, CG dot products, L1/L2 norms).
//
// Two launches: (1) a (blocks_per_row x rows) grid accumulates fixed chunks in double and writes
// one partial per workgroup; (2) one wavefront per row folds its partials (lane-strided, then a
// fixed shuffle tree).  The partition and the combine order depend only on (rows, n), so results
// are bitwise reproducible run to run.
#include "common.hpp"

namespace pxa {
namespace {

inline int blocks_per_row(int64_t rows, int64_t n) {
  int64_t per = (n + 4095) / 4096;  // >= 4 K elements per workgroup
  int64_t cap = rows > 0 ? (4096 + rows - 1) / rows : 1;  // ~16 workgroups per CU in total
  if (cap < 1) cap = 1;
  if (per > cap) per = cap;
  if (per > 1024) per = 1024;
  if (per < 1) per = 1;
  return (int)per;
}

template <typename T, int OP>
__device__ inline double elem(T x, T y) {
  if (OP == PXA_RED_SUMSQ) return (double)x * (double)x;
  if (OP == PXA_RED_DIFFSQ) {
    double d = (double)x - (double)y;
    return d * d;
  }
  if (OP == PXA_RED_DOT) return (double)x * (double)y;
  if (OP == PXA_RED_ABS) return fabs((double)x);
  if (OP == PXA_RED_MAXABS) return fabs((double)x);
  if (OP == PXA_RED_SUM) return (double)x;
  if (OP == PXA_RED_NEGCNT) return x < T(0) ? 1.0 : 0.0;
  if (OP == PXA_RED_MIN || OP == PXA_RED_MAX) return (double)x;
  return 0.0;
}

// identity of the fold (also the value of lanes / threads without elements)
template <int OP>
__device__ inline double ident() {
  if (OP == PXA_RED_MIN) return INFINITY;
  if (OP == PXA_RED_MAX) return -INFINITY;
  return 0.0;
}

template <int OP>
__device__ inline double combine(double a, double b) {
  if (OP == PXA_RED_MAXABS) return a > b ? a : b;
  if (OP == PXA_RED_MIN) return (a < b || a != a) ? a : b;  // NaN in either operand wins
  if (OP == PXA_RED_MAX) return (a > b || a != a) ? a : b;
  return a + b;
}

template <int OP>
__device__ inline double wave_reduce(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = combine<OP>(v, __shfl_down(v, off, 64));
  return v;
}

template <typename T, int OP>
__global__ void __launch_bounds__(kBlock) row_partial_kernel(int64_t n, int nb, const T* __restrict__ x,
                                                             const T* __restrict__ y, double* __restrict__ part) {
  const int64_t row = blockIdx.y;
  const T* xr = x + row * n;
  const T* yr = y ? y + row * n : nullptr;
  int64_t chunk = (n + nb - 1) / nb;
  int64_t lo = (int64_t)blockIdx.x * chunk;
  int64_t hi = lo + chunk < n ? lo + chunk : n;
  double acc = ident<OP>();
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) acc = combine<OP>(acc, elem<T, OP>(xr[i], yr ? yr[i] : T(0)));
  acc = wave_reduce<OP>(acc);
  __shared__ double sw[kBlock / kWave];
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sw[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = sw[0];
    for (int k = 1; k < kBlock / kWave; ++k) r = combine<OP>(r, sw[k]);
    part[row * nb + blockIdx.x] = r;
  }
}

template <int OP>
__global__ void __launch_bounds__(kBlock) row_final_kernel(int64_t rows, int nb, const double* __restrict__ part,
                                                           double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;  // one wavefront per row
  if (r >= rows) return;
  const double* pr = part + r * nb;
  double acc = lane < nb ? pr[lane] : ident<OP>();
  for (int k = lane + 64; k < nb; k += 64) acc = combine<OP>(acc, pr[k]);
  acc = wave_reduce<OP>(acc);
  if (lane == 0) out[r] = acc;
}

template <typename T, int OP>
int launch_reduce(int64_t rows, int64_t n, const void* x, const void* y, double* out, void* work, void* stream) {
  int nb = blocks_per_row(rows, n);
  double* part = (double*)work;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL((row_partial_kernel<T, OP>), dim3(nb, (unsigned)rows), dim3(kBlock), 0, s, n, nb, (const T*)x,
                     (const T*)y, part);
  int e = last_launch_status();
  if (e) return e;
  const int64_t rows_per_block = kBlock / kWave;
  hipLaunchKernelGGL((row_final_kernel<OP>), dim3((unsigned)((rows + rows_per_block - 1) / rows_per_block)), dim3(kBlock),
                     0, s, rows, nb, part, out);
  return last_launch_status();
}


// RelError statistics in one pass (stop.py:353-382): per row, num = sum (x - p)^2 and den = sum p^2,
// plus (optionally) the copy of x the criterion keeps for its next check.  Same partition, per-thread
// order and fold as row_partial_kernel<DIFFSQ> / <SUMSQ> (identical bits), with x and p read once.
template <typename T>
__global__ void __launch_bounds__(kBlock) relerr_partial_kernel(int64_t n, int nb, const T* __restrict__ x,
                                                                const T* __restrict__ p, T* __restrict__ xcopy,
                                                                double* __restrict__ part) {
  const int64_t row = blockIdx.y;
  const T* xr = x + row * n;
  const T* pr = p + row * n;
  T* cr = xcopy ? xcopy + row * n : nullptr;
  int64_t chunk = (n + nb - 1) / nb;
  int64_t lo = (int64_t)blockIdx.x * chunk;
  int64_t hi = lo + chunk < n ? lo + chunk : n;
  double a0 = 0.0, a1 = 0.0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const T xv = xr[i], pv = pr[i];
    a0 = combine<PXA_RED_DIFFSQ>(a0, elem<T, PXA_RED_DIFFSQ>(xv, pv));
    a1 = combine<PXA_RED_SUMSQ>(a1, elem<T, PXA_RED_SUMSQ>(pv, T(0)));
    if (cr) cr[i] = xv;
  }
  a0 = wave_reduce<PXA_RED_SUMSQ>(a0);
  a1 = wave_reduce<PXA_RED_SUMSQ>(a1);
  __shared__ double sw[2][kBlock / kWave];
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    sw[0][w] = a0;
    sw[1][w] = a1;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    double r = sw[threadIdx.x][0];
    for (int k = 1; k < kBlock / kWave; ++k) r = r + sw[threadIdx.x][k];
    part[(int64_t)threadIdx.x * gridDim.y * nb + row * nb + blockIdx.x] = r;
  }
}

template <typename T>
int launch_relerr(int64_t rows, int64_t n, const void* x, const void* p, void* xcopy, double* out, void* work,
                  void* stream) {
  int nb = blocks_per_row(rows, n);
  double* part = (double*)work;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL((relerr_partial_kernel<T>), dim3(nb, (unsigned)rows), dim3(kBlock), 0, s, n, nb, (const T*)x,
                     (const T*)p, (T*)xcopy, part);
  int e = last_launch_status();
  if (e) return e;
  // both statistic rows folded by one launch of the row_final kernel (2 * rows rows of nb partials)
  const int64_t rows_per_block = kBlock / kWave;
  hipLaunchKernelGGL((row_final_kernel<PXA_RED_SUMSQ>), dim3((unsigned)((2 * rows + rows_per_block - 1) / rows_per_block)),
                     dim3(kBlock), 0, s, 2 * rows, nb, part, out);
  return last_launch_status();
}

// Fold of the fused PGD kernel's per-(tile, wavefront) RelError partials (pgd_tv2d.hip: slot t wrote
// part[2 t] = sum (x_new - x)^2 and part[2 t + 1] = sum x^2) into out[0][r] / out[1][r] for each stack row
// r owning slots [r per_row, (r + 1) per_row): one 256-thread workgroup per (statistic, row), thread-strided
// sums with independent loads in flight, then the wave folds and a fixed-order sum of the 4 wave results, so
// the result is deterministic run to run.  (One wavefront per pair was latency-bound: 33 us for the 8 192
// slots of a 2048^2 image, every load a dependent round trip.)
__global__ void __launch_bounds__(kBlock) tile_partials_fold_kernel(int64_t rows, int64_t per_row,
                                                                    const double* __restrict__ part,
                                                                    double* __restrict__ out,
                                                                    unsigned* __restrict__ flags, unsigned seq) {
  __shared__ double red[kBlock / kWave];
  const int64_t q = blockIdx.x;  // q = stat * rows + row
  const int64_t stat = q / rows, r = q - stat * rows;
  const double t = fold_tile_stat<true>(part + 2 * r * per_row + stat, per_row, red);
  if (threadIdx.x == 0) {
    out[q] = t;
    if (flags != nullptr) {  // completion flag of this statistic, ordered after its value system-wide
      __threadfence_system();
      __hip_atomic_store(flags + q, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// General Ln row statistic for the stop criteria (stop.py:222-297 -> pxlg.norm(ord=p)):
// sum |x - y|^p (p > 0), or the count of non-zero entries (p == 0, NumPy's ord=0).  Same partition
// and fold as row_partial_kernel (deterministic).
template <typename T>
__global__ void __launch_bounds__(kBlock) row_pow_kernel(int64_t n, int nb, double p, const T* __restrict__ x,
                                                         const T* __restrict__ y, double* __restrict__ part) {
  const int64_t row = blockIdx.y;
  const T* xr = x + row * n;
  const T* yr = y ? y + row * n : nullptr;
  int64_t chunk = (n + nb - 1) / nb;
  int64_t lo = (int64_t)blockIdx.x * chunk;
  int64_t hi = lo + chunk < n ? lo + chunk : n;
  double acc = 0.0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const double d = fabs((double)xr[i] - (yr ? (double)yr[i] : 0.0));
    acc += p == 0.0 ? (d != 0.0 ? 1.0 : 0.0) : pow(d, p);
  }
  acc = wave_reduce<PXA_RED_SUM>(acc);
  __shared__ double sw[kBlock / kWave];
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sw[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = sw[0];
    for (int k = 1; k < kBlock / kWave; ++k) r = r + sw[k];
    part[row * nb + blockIdx.x] = r;
  }
}

template <typename T>
int launch_pow(int64_t rows, int64_t n, double p, const void* x, const void* y, double* out, void* work, void* stream) {
  int nb = blocks_per_row(rows, n);
  double* part = (double*)work;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL((row_pow_kernel<T>), dim3(nb, (unsigned)rows), dim3(kBlock), 0, s, n, nb, p, (const T*)x,
                     (const T*)y, part);
  int e = last_launch_status();
  if (e) return e;
  const int64_t rows_per_block = kBlock / kWave;
  hipLaunchKernelGGL((row_final_kernel<PXA_RED_SUM>), dim3((unsigned)((rows + rows_per_block - 1) / rows_per_block)),
                     dim3(kBlock), 0, s, rows, nb, part, out);
  return last_launch_status();
}

}  // namespace
}  // namespace pxa

using namespace pxa;

extern "C" {

int pxa_row_reduce_pow(int dtype, int64_t rows, int64_t n, double p, const void* x, const void* y, double* out,
                       void* work, void* stream) {
  PXA_CHECK_ARG(rows >= 0 && n >= 0 && p >= 0.0);
  if (rows == 0) return PXA_OK;
  PXA_CHECK_ARG(rows <= 65535);
  PXA_CHECK_ARG(x != nullptr && out != nullptr && work != nullptr);
  if (n == 0) return (int)hipMemsetAsync(out, 0, rows * sizeof(double), as_stream(stream));
  PXA_DISPATCH(dtype, T, return launch_pow<T>(rows, n, p, x, y, out, work, stream));
}

size_t pxa_row_reduce_workspace_bytes(int64_t rows, int64_t n) {
  if (rows <= 0) return 0;
  return (size_t)rows * (size_t)blocks_per_row(rows, n) * sizeof(double);
}

int pxa_row_reduce(int dtype, int op, int64_t rows, int64_t n, const void* x, const void* y, double* out, void* work,
                   void* stream) {
  PXA_CHECK_ARG(rows >= 0 && n >= 0);
  if (rows == 0) return PXA_OK;
  PXA_CHECK_ARG(rows <= 65535);  // grid.y limit
  PXA_CHECK_ARG(x != nullptr && out != nullptr && work != nullptr);
  if (op == PXA_RED_DIFFSQ || op == PXA_RED_DOT) PXA_CHECK_ARG(y != nullptr);
  if (n == 0) return (int)hipMemsetAsync(out, 0, rows * sizeof(double), as_stream(stream));
#define PXA_RED_CASE(OPC) \
  case OPC:               \
    PXA_DISPATCH(dtype, T, return (launch_reduce<T, OPC>(rows, n, x, y, out, work, stream)));
  switch (op) {
    PXA_RED_CASE(PXA_RED_SUMSQ)
    PXA_RED_CASE(PXA_RED_DIFFSQ)
    PXA_RED_CASE(PXA_RED_DOT)
    PXA_RED_CASE(PXA_RED_ABS)
    PXA_RED_CASE(PXA_RED_MAXABS)
    PXA_RED_CASE(PXA_RED_SUM)
    PXA_RED_CASE(PXA_RED_NEGCNT)
    PXA_RED_CASE(PXA_RED_MIN)
    PXA_RED_CASE(PXA_RED_MAX)
    default:
      return PXA_ERR_ARG;
  }
#undef PXA_RED_CASE
}

int pxa_tile_partials_fold(int64_t rows, int64_t per_row, const double* partials, double* out, uint32_t* flags,
                           uint32_t seq, void* stream) {
  PXA_CHECK_ARG(rows >= 1 && per_row >= 1 && partials != nullptr && out != nullptr);
  PXA_CHECK_ARG(2 * rows <= 0x7fffffff);
  hipLaunchKernelGGL(tile_partials_fold_kernel, dim3((unsigned)(2 * rows)), dim3(kBlock), 0, as_stream(stream), rows,
                     per_row, partials, out, (unsigned*)flags, (unsigned)seq);
  return last_launch_status();
}

int pxa_host_alloc(size_t bytes, void** ptr) {
  PXA_CHECK_ARG(ptr != nullptr && bytes > 0);
  *ptr = nullptr;
  return (int)hipHostMalloc(ptr, bytes, hipHostMallocCoherent | hipHostMallocMapped);
}

int pxa_host_free(void* ptr) { return ptr ? (int)hipHostFree(ptr) : PXA_OK; }

size_t pxa_relerr_stats_workspace_bytes(int64_t rows, int64_t n) { return 2 * pxa_row_reduce_workspace_bytes(rows, n); }

int pxa_relerr_stats(int dtype, int64_t rows, int64_t n, const void* x, const void* x_prev, void* x_copy, double* out,
                     void* work, void* stream) {
  PXA_CHECK_ARG(rows >= 0 && n >= 0);
  if (rows == 0) return PXA_OK;
  PXA_CHECK_ARG(rows <= 65535);  // grid.y limit
  PXA_CHECK_ARG(x != nullptr && x_prev != nullptr && out != nullptr && work != nullptr);
  PXA_CHECK_ARG(x_copy != x && x_copy != x_prev);
  if (n == 0) return (int)hipMemsetAsync(out, 0, 2 * rows * sizeof(double), as_stream(stream));
  PXA_DISPATCH(dtype, T, return launch_relerr<T>(rows, n, x, x_prev, x_copy, out, work, stream));
}

}  // extern "C"
