// CG iteration tail (opt/solver/cg.py:125-153) after A p, in three launches instead of the row-op chain
// (<p, A p> partial + fold, alpha, x update, r update, ||r'||^2 partial + fold, beta, p update, D2H copy):
//   cg_dot    per-block partials of <p, A p> (double)
//   cg_xr     every block folds the <p, A p> partials in the same fixed order, alpha = (T)(rr / pAp) (the
//             float64 division then the cast of the host / row_ratio path), x += alpha p, r -= alpha A p,
//             per-block partials of ||r'||^2
//   cg_p      every block folds the ||r'||^2 partials, beta = (T)(rr' / rr), p = r + beta p; block 0 stores
//             rr' for the next step (device) and into host memory (the stop check's value), then, with
//             `flags`, a completion flag the host polls (coherent host memory, system-scope release)
// One row of the stacked problem per grid.y.  All sums in double with a fixed partition and order, so the
// results are deterministic run to run.  HBM-bound streaming (p, A p read twice; x, r, p written once).
#include "common.hpp"

namespace pxa {
namespace {

// fixed-order fold of the nb partials of row `row` (every thread gets the same bits): s = 0 + part[0] + part[1]
// + ... in order.  The partials are loaded 64 at a time, one per lane, and broadcast lane by lane into the
// sequential sum, instead of one dependent L2 round trip per partial.
__device__ inline double fold(const double* __restrict__ part, int64_t row, int nb) {
  const int lane = threadIdx.x & 63;
  const double* pr = part + row * nb;
  double s = 0.0;
  for (int k0 = 0; k0 < nb; k0 += 64) {
    const double v = k0 + lane < nb ? pr[k0 + lane] : 0.0;
    const int m = nb - k0 < 64 ? nb - k0 : 64;
    for (int j = 0; j < m; ++j) s += __shfl(v, j, 64);
  }
  return s;
}

template <typename T>
__global__ void __launch_bounds__(kBlock) cg_dot_kernel(int64_t n, const T* __restrict__ p, const T* __restrict__ ap,
                                                        double* __restrict__ part) {
  __shared__ double sh[kBlock / 64];
  const int64_t row = blockIdx.y;
  const int64_t chunk = (n + gridDim.x - 1) / gridDim.x, lo = blockIdx.x * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  const T* pr = p + row * n;
  const T* ar = ap + row * n;
  double acc = 0.0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) acc = fma((double)pr[i], (double)ar[i], acc);
  const double s = cg_block_sum(acc, sh);
  if (threadIdx.x == 0) part[row * gridDim.x + blockIdx.x] = s;
}

// The streaming loads of a thread's elements lo + t, lo + t + kBlock, ... are issued kCgBatch at a time, the
// first batch before the partial fold (alpha / beta do not gate them); the per-thread order of the sums is the
// element order, as in cg_dot.
constexpr int kCgBatch = 4;

template <typename T>
__global__ void __launch_bounds__(kBlock) cg_xr_kernel(int64_t n, const double* __restrict__ rr,
                                                       const double* __restrict__ part_pap, const T* __restrict__ p,
                                                       const T* __restrict__ ap, T* __restrict__ x, T* __restrict__ r,
                                                       double* __restrict__ part_rr) {
  __shared__ double sh[kBlock / 64];
  const int64_t row = blockIdx.y;
  const int64_t chunk = (n + gridDim.x - 1) / gridDim.x, lo = blockIdx.x * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  const T* pr = p + row * n;
  const T* ar = ap + row * n;
  T* xr = x + row * n;
  T* rw = r + row * n;
  T pv[kCgBatch], av[kCgBatch], xv[kCgBatch], rv[kCgBatch];
  auto load = [&](int64_t ib) {
#pragma unroll
    for (int k = 0; k < kCgBatch; ++k) {
      const int64_t i = ib + (int64_t)k * kBlock;
      if (i < hi) {
        pv[k] = pr[i];
        av[k] = ar[i];
        xv[k] = xr[i];
        rv[k] = rw[i];
      }
    }
  };
  const int64_t i0 = lo + threadIdx.x;
  load(i0);
  const T alpha = (T)(rr[row] / fold(part_pap, row, gridDim.x));
  double acc = 0.0;
  for (int64_t ib = i0; ib < hi; ib += (int64_t)kCgBatch * kBlock) {
    if (ib != i0) load(ib);
#pragma unroll
    for (int k = 0; k < kCgBatch; ++k) {
      const int64_t i = ib + (int64_t)k * kBlock;
      if (i < hi) {
        xr[i] = fma(alpha, pv[k], xv[k]);          // x += alpha p
        const T rn = fma(-alpha, av[k], rv[k]);    // r -= alpha A p
        rw[i] = rn;
        acc = fma((double)rn, (double)rn, acc);
      }
    }
  }
  const double s = cg_block_sum(acc, sh);
  if (threadIdx.x == 0) part_rr[row * gridDim.x + blockIdx.x] = s;
}

template <typename T>
__global__ void __launch_bounds__(kBlock) cg_p_kernel(int64_t n, const double* __restrict__ rr,
                                                      const double* __restrict__ part_rr, const T* __restrict__ r,
                                                      T* __restrict__ p, double* __restrict__ rr_out,
                                                      double* __restrict__ rr_host, unsigned* __restrict__ flags,
                                                      unsigned seq) {
  const int64_t row = blockIdx.y;
  const int64_t chunk = (n + gridDim.x - 1) / gridDim.x, lo = blockIdx.x * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  const T* rw = r + row * n;
  T* pw = p + row * n;
  T rv[kCgBatch], pv[kCgBatch];
  auto load = [&](int64_t ib) {
#pragma unroll
    for (int k = 0; k < kCgBatch; ++k) {
      const int64_t i = ib + (int64_t)k * kBlock;
      if (i < hi) {
        rv[k] = rw[i];
        pv[k] = pw[i];
      }
    }
  };
  const int64_t i0 = lo + threadIdx.x;
  load(i0);
  const double rn = fold(part_rr, row, gridDim.x);
  const T beta = (T)(rn / rr[row]);
  for (int64_t ib = i0; ib < hi; ib += (int64_t)kCgBatch * kBlock) {
    if (ib != i0) load(ib);
#pragma unroll
    for (int k = 0; k < kCgBatch; ++k) {
      const int64_t i = ib + (int64_t)k * kBlock;
      if (i < hi) pw[i] = fma(beta, pv[k], rv[k]);  // p = r + beta p
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    rr_out[row] = rn;
    if (rr_host) rr_host[row] = rn;
    if (flags) {  // the stop check polls this flag instead of waiting for a stream event
      __threadfence_system();
      __hip_atomic_store(flags + row, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

}  // namespace
}  // namespace pxa

using namespace pxa;

namespace {
int cg_update(int dtype, int64_t rows, int64_t n, void* x, void* r, void* p, const void* ap, const double* rr,
              double* rr_out, double* rr_host, uint32_t* flags, uint32_t seq, void* work, bool have_pap, void* stream) {
  PXA_CHECK_ARG(rows >= 1 && rows <= 65535 && n >= 1);
  PXA_CHECK_ARG(x && r && p && ap && rr && rr_out && work && rr_out != rr);
  hipStream_t st = as_stream(stream);
  const int nb = cg_blocks(n);
  double* part_pap = (double*)work;
  double* part_rr = part_pap + rows * kCgBlocks;
  const dim3 grid((unsigned)nb, (unsigned)rows);
  PXA_DISPATCH(dtype, T, {
    int e = 0;
    if (!have_pap) {
      hipLaunchKernelGGL((cg_dot_kernel<T>), grid, dim3(kBlock), 0, st, n, (const T*)p, (const T*)ap, part_pap);
      e = last_launch_status();
      if (e) return e;
    }
    hipLaunchKernelGGL((cg_xr_kernel<T>), grid, dim3(kBlock), 0, st, n, rr, part_pap, (const T*)p, (const T*)ap,
                       (T*)x, (T*)r, part_rr);
    e = last_launch_status();
    if (e) return e;
    hipLaunchKernelGGL((cg_p_kernel<T>), grid, dim3(kBlock), 0, st, n, rr, part_rr, (const T*)r, (T*)p, rr_out,
                       rr_host, (unsigned*)flags, (unsigned)seq);
    return last_launch_status();
  });
}
}  // namespace

extern "C" {

size_t pxa_cg_update_workspace_bytes(int64_t rows) { return rows > 0 ? (size_t)rows * 2 * kCgBlocks * sizeof(double) : 0; }

int pxa_cg_update(int dtype, int64_t rows, int64_t n, void* x, void* r, void* p, const void* ap, const double* rr,
                  double* rr_out, double* rr_host, uint32_t* flags, uint32_t seq, void* work, void* stream) {
  return cg_update(dtype, rows, n, x, r, p, ap, rr, rr_out, rr_host, flags, seq, work, false, stream);
}

int pxa_cg_update_tail(int dtype, int64_t rows, int64_t n, void* x, void* r, void* p, const void* ap, const double* rr,
                       double* rr_out, double* rr_host, uint32_t* flags, uint32_t seq, void* work, void* stream) {
  return cg_update(dtype, rows, n, x, r, p, ap, rr, rr_out, rr_host, flags, seq, work, true, stream);
}

int pxa_cg_update_xr(int dtype, int64_t rows, int64_t n, void* x, void* r, const void* p, const void* ap, const double* rr,
                     void* work, void* stream) {
  PXA_CHECK_ARG(rows >= 1 && rows <= 65535 && n >= 1);
  PXA_CHECK_ARG(x && r && p && ap && rr && work);
  hipStream_t st = as_stream(stream);
  const int nb = cg_blocks(n);
  double* part_pap = (double*)work;
  double* part_rr = part_pap + rows * kCgBlocks;
  PXA_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((cg_xr_kernel<T>), dim3((unsigned)nb, (unsigned)rows), dim3(kBlock), 0, st, n, rr, part_pap,
                       (const T*)p, (const T*)ap, (T*)x, (T*)r, part_rr);
    return last_launch_status();
  });
}

}  // extern "C"
