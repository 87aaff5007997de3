// Array primitives of the operator algebra and of the NumPy-named `xp` shim: strided 2-D copies /
// accumulations (block-operator concatenation and sums, blocks.py:660-679, 838-860; broadcasts),
// element-wise unary / binary maps, where, dtype casts, diagonal writes and transposes.  They keep
// every array operation of the product path inside this library (no torch arithmetic).
//
// All are HBM-bound streaming kernels: 16-B vectors where the rows allow it, grid-stride loops.
#include "common.hpp"

namespace pxa {
namespace {

// dst[r * ldd + i] = src[r * lds + i] (acc 0), dst + src (acc 1), 0 + src (acc 2)     r < rows, i < n
template <typename T, bool VEC>
__global__ void __launch_bounds__(kBlock) copy2d_kernel(int64_t rows, int64_t n, const T* src, int64_t lds, int64_t sci,
                                                        T* dst, int64_t ldd, int acc) {
  constexpr int V = VEC ? kVecN<T> : 1;
  using VT = typename Vec4<T>::type;
  const int64_t nv = n / V;
  for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
    const T* s = src + r * lds;
    T* d = dst + r * ldd;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
      if constexpr (VEC) {
        VT v = reinterpret_cast<const VT*>(s)[i];
        if (acc == 2) {  // 0 + s: the first term of a Python sum() (turns -0.0 into +0.0, as the reference)
          T* pv = reinterpret_cast<T*>(&v);
#pragma unroll
          for (int k = 0; k < V; ++k) pv[k] = T(0) + pv[k];
        } else if (acc) {
          const VT o = reinterpret_cast<const VT*>(d)[i];
          T* pv = reinterpret_cast<T*>(&v);
          const T* po = reinterpret_cast<const T*>(&o);
#pragma unroll
          for (int k = 0; k < V; ++k) pv[k] = po[k] + pv[k];
        }
        reinterpret_cast<VT*>(d)[i] = v;
      } else {
        const T v = s[i * sci];
        d[i] = acc == 2 ? T(0) + v : (acc ? d[i] + v : v);
      }
    }
  }
}

enum UnaryOp { kSqrt = 0, kSign = 1, kAbs = 2, kNeg = 3, kSquare = 4, kReciprocal = 5, kPosInf = 6 };

template <typename T>
__device__ inline T unary(int op, T x) {
  switch (op) {
    case kSqrt:
      return sqrt(x);
    case kSign:  // numpy.sign: -1 / +0 / +1 (also for -0.0), NaN stays NaN
      return x > T(0) ? T(1) : (x < T(0) ? T(-1) : (x == T(0) ? T(0) : x));
    case kAbs:
      return fabs(x);
    case kNeg:
      return -x;
    case kSquare:
      return x * x;
    case kReciprocal:
      return T(1) / x;
    default:  // indicator value of a violated constraint count: +inf if x > 0 else 0
      return x > T(0) ? T(INFINITY) : T(0);
  }
}

enum BinaryOp { kFmax = 0, kFmin = 1, kAdd = 2, kSub = 3, kMul = 4, kDiv = 5, kMaximum = 6, kMinimum = 7, kPow = 8 };

template <typename T>
__device__ inline T binary(int op, T a, T b) {
  switch (op) {
    case kFmax:  // numpy.fmax: NaN-ignoring
      return fmax(a, b);
    case kFmin:
      return fmin(a, b);
    case kAdd:
      return a + b;
    case kSub:
      return a - b;
    case kMul:
      return a * b;
    case kDiv:
      return a / b;
    case kMaximum:  // numpy.maximum: NaN-propagating
      return (a != a || b != b) ? a + b : (a > b ? a : b);
    case kMinimum:
      return (a != a || b != b) ? a + b : (a < b ? a : b);
    default:
      return pow(a, b);
  }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) unary_kernel(int64_t n, int op, const T* x, T* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = unary<T>(op, x[i]);
}

// x / y: arrays, or NULL for the broadcast scalars xs / ys
template <typename T>
__global__ void __launch_bounds__(kBlock) binary_kernel(int64_t n, int op, const T* x, T xs, const T* y, T ys,
                                                        T* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = binary<T>(op, x ? x[i] : xs, y ? y[i] : ys);
}

template <typename T>
__global__ void __launch_bounds__(kBlock) where_kernel(int64_t n, const unsigned char* cond, const T* x, T xs,
                                                       const T* y, T ys, T* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = cond[i] ? (x ? x[i] : xs) : (y ? y[i] : ys);
}

template <typename TI, typename TO>
__global__ void __launch_bounds__(kBlock) cast_kernel(int64_t n, const TI* x, TO* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (TO)x[i];
}

template <typename T>
__global__ void __launch_bounds__(kBlock) set_diag_kernel(int64_t rows, int64_t ld, int64_t off, T v, T* out) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x)
    out[r * ld + off + r] = v;
}

// dst (cols, rows) = src (rows, cols)^T through a 32 x 33 LDS tile (conflict-free column reads)
template <typename T>
__global__ void __launch_bounds__(256) transpose_kernel(int64_t rows, int64_t cols, const T* src, T* dst) {
  __shared__ T tile[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8 threads
  for (int64_t bi = blockIdx.y; bi * 32 < rows; bi += gridDim.y) {
    for (int64_t bj = blockIdx.x; bj * 32 < cols; bj += gridDim.x) {
      const int64_t r0 = bi * 32, c0 = bj * 32;
#pragma unroll
      for (int k = 0; k < 32; k += 8) {
        const int64_t r = r0 + ty + k, c = c0 + tx;
        if (r < rows && c < cols) tile[ty + k][tx] = src[r * cols + c];
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 32; k += 8) {
        const int64_t c = c0 + ty + k, r = r0 + tx;
        if (r < rows && c < cols) dst[c * rows + r] = tile[tx][ty + k];
      }
      __syncthreads();
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) isnan_kernel(int64_t n, const T* x, unsigned char* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = x[i] != x[i] ? 1 : 0;
}

// out[0] = any(x) (mode 0) or all(x) (mode 1) over n bytes; out must be pre-set by the caller to the
// neutral value (0 for any, 1 for all); every thread that sees the deciding value stores it (idempotent)
__global__ void __launch_bounds__(kBlock) bool_reduce_kernel(int64_t n, int mode, const unsigned char* x,
                                                             unsigned char* out) {
  bool hit = false;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    hit |= mode == 0 ? (x[i] != 0) : (x[i] == 0);
  if (hit) out[0] = mode == 0 ? 1 : 0;
}

// y[r, j] = x[r, idx[j]]  (SubSample.apply)            r < rows, j < m
template <typename T>
__global__ void __launch_bounds__(kBlock) gather_cols_kernel(int64_t rows, int64_t n, const T* x, int64_t m,
                                                             const int64_t* idx, T* y) {
  for (int64_t r = blockIdx.y; r < rows; r += gridDim.y)
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x)
      y[r * m + j] = x[r * n + idx[j]];
}

// out[r, idx[j]] = y[r, j] over an out the caller zero-filled (SubSample.adjoint); idx unique
template <typename T>
__global__ void __launch_bounds__(kBlock) scatter_cols_kernel(int64_t rows, int64_t m, const T* y, int64_t n,
                                                              const int64_t* idx, T* out) {
  for (int64_t r = blockIdx.y; r < rows; r += gridDim.y)
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x)
      out[r * n + idx[j]] = y[r * m + j];
}

inline unsigned gy(int64_t rows) { return (unsigned)(rows < 1 ? 1 : (rows > 65535 ? 65535 : rows)); }

// Directional contraction of a stacked derivative output (Sum o DiagonalOp o {Gradient, Hessian},
// diff.py:1938-2759).  apply:   y[s][g][p] = sum_{j < J} w[g][j][p] * x[s][j % K][p]
//                    adjoint: y[s][k][p] = sum_{g < G} sum_{j % K == k} w[g][j][p] * x[s][g][p]
// w is (G, J, N) (wp = 1) or (G, J) broadcast over the pixels (wp = 0).  Each product is rounded, then
// the terms are added in order (j, then g), like the reference's DiagonalOp followed by numpy.sum over
// the leading axes (no fma contraction).  One thread per (s, p), grid-stride.
template <typename T, bool ADJ>
__global__ void __launch_bounds__(kBlock) dir_contract_kernel(int64_t S, int64_t G, int64_t J, int64_t K, int64_t N,
                                                              const T* __restrict__ w, int64_t wp,
                                                              const T* __restrict__ x, T* __restrict__ y) {
#pragma clang fp contract(off)
  const int64_t total = S * N;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t sidx = q / N, p = q - sidx * N;
    const int64_t pw = wp ? p : 0, ldw = wp ? N : 1;
    if constexpr (!ADJ) {
      const T* xs = x + sidx * K * N + p;
      T* ys = y + sidx * G * N + p;
      for (int64_t g = 0; g < G; ++g) {
        T acc = T(0);
        for (int64_t j = 0; j < J; ++j) {
          const T t = w[(g * J + j) * ldw + pw] * xs[(j % K) * N];
          acc = j == 0 ? t : acc + t;
        }
        ys[g * N] = acc;
      }
    } else {
      const T* xs = x + sidx * G * N + p;
      T* ys = y + sidx * K * N + p;
      for (int64_t k = 0; k < K; ++k) {
        T acc = T(0);
        bool first = true;
        for (int64_t g = 0; g < G; ++g)
          for (int64_t j = k; j < J; j += K) {
            const T t = w[(g * J + j) * ldw + pw] * xs[g * N];
            acc = first ? t : acc + t;
            first = false;
          }
        ys[k * N] = acc;
      }
    }
  }
}

}  // namespace
}  // namespace pxa

using namespace pxa;

extern "C" {

int pxa_copy2d(int dtype, int64_t rows, int64_t n, const void* src, int64_t lds, int64_t src_col_stride, void* dst,
               int64_t ldd, int accumulate, void* stream) {
  PXA_CHECK_ARG(rows >= 0 && n >= 0 && lds >= 0 && ldd >= n && (src_col_stride == 0 || src_col_stride == 1));
  PXA_CHECK_ARG(accumulate >= 0 && accumulate <= 2);
  if (rows == 0 || n == 0) return PXA_OK;
  PXA_CHECK_ARG(src != nullptr && dst != nullptr);
  PXA_DISPATCH(dtype, T, {
    constexpr int V = kVecN<T>;
    const bool vec = src_col_stride == 1 && (n % V == 0) && (lds % V == 0) && (ldd % V == 0) && aligned16(src) &&
                     aligned16(dst);
    const int64_t items = vec ? n / V : n;
    int gx = (int)((items + kBlock - 1) / kBlock);
    const unsigned gyv = gy(rows);
    int64_t cap = (kMaxGrid + gyv - 1) / gyv;
    if (gx > cap) gx = (int)cap;
    if (gx < 1) gx = 1;
    if (vec)
      hipLaunchKernelGGL((copy2d_kernel<T, true>), dim3(gx, gyv), dim3(kBlock), 0, as_stream(stream), rows, n,
                         (const T*)src, lds, (int64_t)1, (T*)dst, ldd, accumulate);
    else
      hipLaunchKernelGGL((copy2d_kernel<T, false>), dim3(gx, gyv), dim3(kBlock), 0, as_stream(stream), rows, n,
                         (const T*)src, lds, src_col_stride, (T*)dst, ldd, accumulate);
    return last_launch_status();
  });
}

int pxa_unary(int dtype, int op, int64_t n, const void* x, void* out, void* stream) {
  PXA_CHECK_ARG(n >= 0 && op >= 0 && op <= kPosInf);
  if (n == 0) return PXA_OK;
  PXA_CHECK_ARG(x != nullptr && out != nullptr);
  PXA_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((unary_kernel<T>), dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), n, op, (const T*)x,
                       (T*)out);
    return last_launch_status();
  });
}

int pxa_binary(int dtype, int op, int64_t n, const void* x, double xs, const void* y, double ys, void* out,
               void* stream) {
  PXA_CHECK_ARG(n >= 0 && op >= 0 && op <= kPow);
  if (n == 0) return PXA_OK;
  PXA_CHECK_ARG(out != nullptr);
  PXA_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((binary_kernel<T>), dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), n, op, (const T*)x,
                       (T)xs, (const T*)y, (T)ys, (T*)out);
    return last_launch_status();
  });
}

int pxa_where(int dtype, int64_t n, const void* cond, const void* x, double xs, const void* y, double ys, void* out,
              void* stream) {
  PXA_CHECK_ARG(n >= 0);
  if (n == 0) return PXA_OK;
  PXA_CHECK_ARG(cond != nullptr && out != nullptr);
  PXA_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((where_kernel<T>), dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), n,
                       (const unsigned char*)cond, (const T*)x, (T)xs, (const T*)y, (T)ys, (T*)out);
    return last_launch_status();
  });
}

int pxa_cast(int dtype_in, int dtype_out, int64_t n, const void* x, void* out, void* stream) {
  PXA_CHECK_ARG(n >= 0);
  if (n == 0) return PXA_OK;
  PXA_CHECK_ARG(x != nullptr && out != nullptr);
  PXA_DISPATCH(dtype_in, TI, {
    PXA_DISPATCH(dtype_out, TO, {
      hipLaunchKernelGGL((cast_kernel<TI, TO>), dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), n, (const TI*)x,
                         (TO*)out);
      return last_launch_status();
    });
  });
}

int pxa_set_diag(int dtype, int64_t rows, int64_t ld, int64_t off, double value, void* out, void* stream) {
  PXA_CHECK_ARG(rows >= 0 && off >= 0 && ld >= 0);
  if (rows == 0) return PXA_OK;
  PXA_CHECK_ARG(out != nullptr);
  PXA_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((set_diag_kernel<T>), dim3(grid_for(rows)), dim3(kBlock), 0, as_stream(stream), rows, ld, off,
                       (T)value, (T*)out);
    return last_launch_status();
  });
}

int pxa_transpose(int dtype, int64_t rows, int64_t cols, const void* src, void* dst, void* stream) {
  PXA_CHECK_ARG(rows >= 0 && cols >= 0);
  if (rows == 0 || cols == 0) return PXA_OK;
  PXA_CHECK_ARG(src != nullptr && dst != nullptr && src != dst);
  PXA_DISPATCH(dtype, T, {
    const int64_t bx = (cols + 31) / 32, by = (rows + 31) / 32;
    dim3 grid((unsigned)(bx > 1024 ? 1024 : bx), (unsigned)(by > 1024 ? 1024 : by));
    hipLaunchKernelGGL((transpose_kernel<T>), grid, dim3(256), 0, as_stream(stream), rows, cols, (const T*)src, (T*)dst);
    return last_launch_status();
  });
}

int pxa_isnan(int dtype, int64_t n, const void* x, void* out, void* stream) {
  PXA_CHECK_ARG(n >= 0);
  if (n == 0) return PXA_OK;
  PXA_CHECK_ARG(x != nullptr && out != nullptr);
  PXA_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((isnan_kernel<T>), dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), n, (const T*)x,
                       (unsigned char*)out);
    return last_launch_status();
  });
}

int pxa_bool_reduce(int64_t n, int mode, const void* x, void* out, void* stream) {
  PXA_CHECK_ARG(n >= 0 && (mode == 0 || mode == 1) && out != nullptr);
  hipError_t e = hipMemsetAsync(out, mode == 0 ? 0 : 1, 1, as_stream(stream));
  if (e != hipSuccess) return (int)e;
  if (n == 0) return PXA_OK;
  PXA_CHECK_ARG(x != nullptr);
  hipLaunchKernelGGL(bool_reduce_kernel, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), n, mode,
                     (const unsigned char*)x, (unsigned char*)out);
  return last_launch_status();
}

int pxa_gather_cols(int dtype, int64_t rows, int64_t n, const void* x, int64_t m, const int64_t* idx_dev, void* y,
                    void* stream) {
  PXA_CHECK_ARG(rows >= 0 && n >= 0 && m >= 0);
  if (rows == 0 || m == 0) return PXA_OK;
  PXA_CHECK_ARG(x != nullptr && y != nullptr && idx_dev != nullptr && n > 0);
  PXA_DISPATCH(dtype, T, {
    const unsigned gyv = gy(rows);
    int64_t gx = (m + kBlock - 1) / kBlock, cap = (kMaxGrid + gyv - 1) / gyv;
    gx = gx > cap ? cap : gx;
    hipLaunchKernelGGL((gather_cols_kernel<T>), dim3((unsigned)gx, gyv), dim3(kBlock), 0, as_stream(stream), rows, n,
                       (const T*)x, m, idx_dev, (T*)y);
    return last_launch_status();
  });
}

int pxa_scatter_cols(int dtype, int64_t rows, int64_t m, const void* y, int64_t n, const int64_t* idx_dev, void* out,
                     void* stream) {
  PXA_CHECK_ARG(rows >= 0 && n >= 0 && m >= 0);
  if (rows == 0 || n == 0) return PXA_OK;
  PXA_CHECK_ARG(out != nullptr);
  PXA_DISPATCH(dtype, T, {
    hipError_t e = hipMemsetAsync(out, 0, (size_t)(rows * n) * sizeof(T), as_stream(stream));
    if (e != hipSuccess) return (int)e;
    if (m == 0) return PXA_OK;
    PXA_CHECK_ARG(y != nullptr && idx_dev != nullptr);
    const unsigned gyv = gy(rows);
    int64_t gx = (m + kBlock - 1) / kBlock, cap = (kMaxGrid + gyv - 1) / gyv;
    gx = gx > cap ? cap : gx;
    hipLaunchKernelGGL((scatter_cols_kernel<T>), dim3((unsigned)gx, gyv), dim3(kBlock), 0, as_stream(stream), rows, m,
                       (const T*)y, n, idx_dev, (T*)out);
    return last_launch_status();
  });
}

int pxa_dir_contract(int dtype, int64_t S, int64_t G, int64_t J, int64_t K, int64_t N, const void* w, int64_t wp,
                     const void* x, void* y, int adjoint, void* stream) {
  PXA_CHECK_ARG(S >= 0 && G >= 1 && K >= 1 && J >= K && J % K == 0 && N >= 0 && (wp == 0 || wp == 1));
  PXA_CHECK_ARG(w && x && y && x != y);
  if (S == 0 || N == 0) return PXA_OK;
  const int grid = grid_for(S * N);
  hipStream_t st = as_stream(stream);
  PXA_DISPATCH(dtype, T, {
    if (adjoint)
      hipLaunchKernelGGL((dir_contract_kernel<T, true>), dim3(grid), dim3(kBlock), 0, st, S, G, J, K, N, (const T*)w, wp,
                         (const T*)x, (T*)y);
    else
      hipLaunchKernelGGL((dir_contract_kernel<T, false>), dim3(grid), dim3(kBlock), 0, st, S, G, J, K, N, (const T*)w, wp,
                         (const T*)x, (T*)y);
    return last_launch_status();
  });
}

}  // extern "C"
