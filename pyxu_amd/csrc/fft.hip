// FFT LinOp (operator/linop/fft/fft.py:257-379): multi-dimensional DFT over any subset of axes of a
// stack of complex arrays (interleaved re/im, the reference's view_as_real layout).
//   apply   = fftn(x, axes, norm="backward")   (exponent sign -, unnormalised)
//   adjoint = ifftn(x, axes, norm="forward")   (exponent sign +, unnormalised)
//
// One pass per transformed axis, each pass in place on the output: a workgroup loads LPB whole lines
// of the axis into LDS, runs a mixed-radix Stockham autosort FFT there (radices 8, 4, 2, 3, 5, 7;
// stage s with radix R and span Ns: v[r] = src[j + r n/R] w^(r (j mod Ns)), v = DFT_R(v),
// dst[(j div Ns) Ns R + (j mod Ns) + r Ns] = v[r]; the result is in natural order), and writes the
// lines back.  Strided axes gather LPB adjacent lines per workgroup so that every global access is
// coalesced across lines; the contiguous axis reads whole lines.  Lengths with a prime factor > 7 use
// an exact O(n^2) DFT of the LDS-resident line (twiddle index j k mod n in integers).
// Twiddles: sincospi of an exact rational (2 r k / (Ns R)), fp32 or fp64 like the data.
#include "common.hpp"

namespace pxa {
namespace {

constexpr int kFftThreads = 256;
constexpr int kMaxStages = 24;
constexpr size_t kFftLds = 64 * 1024;  // two LDS buffers of lines (2 workgroups per CU)

template <typename T>
struct Cx {
  T re, im;
};
template <typename T>
__device__ inline Cx<T> cmul(Cx<T> a, Cx<T> b) {
  return Cx<T>{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
template <typename T>
__device__ inline Cx<T> cadd(Cx<T> a, Cx<T> b) {
  return Cx<T>{a.re + b.re, a.im + b.im};
}
template <typename T>
__device__ inline Cx<T> csub(Cx<T> a, Cx<T> b) {
  return Cx<T>{a.re - b.re, a.im - b.im};
}
// multiply by -i (forward) or +i (inverse)
template <typename T, bool INV>
__device__ inline Cx<T> mul_mi(Cx<T> a) {
  return INV ? Cx<T>{-a.im, a.re} : Cx<T>{a.im, -a.re};
}

__device__ inline void sc_pi(float x, float* s, float* c) { sincospif(x, s, c); }
__device__ inline void sc_pi(double x, double* s, double* c) { sincospi(x, s, c); }

// e^{sign 2 pi i num / den}
template <typename T, bool INV>
__device__ inline Cx<T> twiddle(int num, int den) {
  T s, c;
  sc_pi((T)(2 * num) / (T)den, &s, &c);
  return Cx<T>{c, INV ? s : -s};
}

template <typename T, bool INV>
__device__ inline void dft2(Cx<T>* v) {
  const Cx<T> a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}
template <typename T, bool INV>
__device__ inline void dft4(Cx<T>* v) {
  const Cx<T> t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
  const Cx<T> t2 = cadd(v[1], v[3]), t3 = mul_mi<T, INV>(csub(v[1], v[3]));
  v[0] = cadd(t0, t2);
  v[2] = csub(t0, t2);
  v[1] = cadd(t1, t3);
  v[3] = csub(t1, t3);
}
template <typename T, bool INV>
__device__ inline void dft8(Cx<T>* v) {
  Cx<T> e[4] = {v[0], v[2], v[4], v[6]}, o[4] = {v[1], v[3], v[5], v[7]};
  dft4<T, INV>(e);
  dft4<T, INV>(o);
  const T h = T(0.70710678118654752440);
  // W8^k o_k, W8 = e^{-+ i pi / 4}
  const Cx<T> w1 = INV ? Cx<T>{h, h} : Cx<T>{h, -h};
  const Cx<T> w3 = INV ? Cx<T>{-h, h} : Cx<T>{-h, -h};
  Cx<T> p[4] = {o[0], cmul(o[1], w1), mul_mi<T, INV>(o[2]), cmul(o[3], w3)};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = cadd(e[k], p[k]);
    v[k + 4] = csub(e[k], p[k]);
  }
}
// e^{-+2 pi i m / R} for the odd radices, as literal constants (no sincos per butterfly)
template <typename T, bool INV, int R>
__device__ inline Cx<T> root(int m) {
  constexpr double c3[2] = {-0.5, 0.86602540378443864676};
  constexpr double c5[4] = {0.30901699437494742410, 0.95105651629515357212, -0.80901699437494742410,
                            0.58778525229247312917};
  constexpr double c7[6] = {0.62348980185873353053, 0.78183148246802980871, -0.22252093395631440429,
                            0.97492791218182360702, -0.90096886790241912624, 0.43388373911755812048};
  if (m == 0) return Cx<T>{T(1), T(0)};
  const int h = m <= R / 2 ? m : R - m;  // cos symmetric, sin antisymmetric
  const double* t = R == 3 ? c3 : (R == 5 ? c5 : c7);
  const T c = (T)t[2 * (h - 1)];
  T sn = (T)t[2 * (h - 1) + 1];
  if (m > R / 2) sn = -sn;
  return Cx<T>{c, INV ? sn : -sn};
}

// odd prime radix: direct DFT with the R roots of unity
template <typename T, bool INV, int R>
__device__ inline void dft_odd(Cx<T>* v) {
  Cx<T> w[R];
#pragma unroll
  for (int m = 0; m < R; ++m) w[m] = root<T, INV, R>(m);
  Cx<T> out[R];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    Cx<T> acc = v[0];
#pragma unroll
    for (int m = 1; m < R; ++m) acc = cadd(acc, cmul(v[m], w[(m * q) % R]));
    out[q] = acc;
  }
#pragma unroll
  for (int q = 0; q < R; ++q) v[q] = out[q];
}

struct FftPlan {
  int64_t n, inner, lines;  // axis length, stride of the axis (elements), number of lines
  int lpb;                   // lines per workgroup
  int nst;
  int radix[kMaxStages];
};

__device__ inline int64_t line_base(int64_t line, int64_t n, int64_t inner) {
  const int64_t o = line / inner;
  return o * n * inner + (line - o * inner);
}

template <typename T, bool INV, int R>
__device__ inline void stage(const Cx<T>* src, Cx<T>* dst, int n, int ns, int lpb) {
  const int nr = n / R;
  for (int b = threadIdx.x; b < lpb * nr; b += kFftThreads) {
    const int l = b / nr, j = b - l * nr;
    const int k = j % ns;
    const Cx<T>* s = src + l * n;
    Cx<T>* d = dst + l * n;
    Cx<T> v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = s[j + r * nr];
    if (ns > 1) {  // w^r from one sincospi: w^1, then successive products (error ~ r ulp)
      const Cx<T> w1 = twiddle<T, INV>(k, ns * R);
      Cx<T> w = w1;
#pragma unroll
      for (int r = 1; r < R; ++r) {
        v[r] = cmul(v[r], w);
        if (r + 1 < R) w = cmul(w, w1);
      }
    }
    if constexpr (R == 2) dft2<T, INV>(v);
    else if constexpr (R == 4) dft4<T, INV>(v);
    else if constexpr (R == 8) dft8<T, INV>(v);
    else dft_odd<T, INV, R>(v);
    const int id = (j / ns) * ns * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) d[id + r * ns] = v[r];
  }
}

// load / store of LPB lines between global (interleaved complex) and LDS (line-major)
template <typename T>
__device__ inline void move_lines(const FftPlan& p, int64_t line0, int nl, const Cx<T>* g, Cx<T>* lds, bool to_lds) {
  const int n = (int)p.n;
  if (p.inner == 1) {  // contiguous axis: the lines are consecutive blocks
    Cx<T>* gl = const_cast<Cx<T>*>(g) + line0 * n;
    for (int i = threadIdx.x; i < nl * n; i += kFftThreads) {
      if (to_lds) lds[i] = gl[i];
      else gl[i] = lds[i];
    }
  } else {  // strided axis: adjacent lines are adjacent in memory at each position m
    for (int i = threadIdx.x; i < nl * n; i += kFftThreads) {
      const int m = i / nl, l = i - m * nl;
      const int64_t off = line_base(line0 + l, p.n, p.inner) + (int64_t)m * p.inner;
      if (to_lds) lds[l * n + m] = g[off];
      else const_cast<Cx<T>*>(g)[off] = lds[l * n + m];
    }
  }
}

template <typename T, bool INV>
__global__ void __launch_bounds__(kFftThreads) fft_stockham_kernel(FftPlan p, const Cx<T>* __restrict__ src,
                                                                   Cx<T>* dst) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int n = (int)p.n;
  const int64_t line0 = (int64_t)blockIdx.x * p.lpb;
  const int nl = (int)((p.lines - line0) < p.lpb ? (p.lines - line0) : p.lpb);
  Cx<T>* b0 = reinterpret_cast<Cx<T>*>(smem_raw);
  Cx<T>* b1 = b0 + (size_t)p.lpb * n;
  move_lines<T>(p, line0, nl, src, b0, true);
  __syncthreads();
  int ns = 1;
  for (int s = 0; s < p.nst; ++s) {
    const int R = p.radix[s];
    switch (R) {
      case 8: stage<T, INV, 8>(b0, b1, n, ns, nl); break;
      case 4: stage<T, INV, 4>(b0, b1, n, ns, nl); break;
      case 2: stage<T, INV, 2>(b0, b1, n, ns, nl); break;
      case 3: stage<T, INV, 3>(b0, b1, n, ns, nl); break;
      case 5: stage<T, INV, 5>(b0, b1, n, ns, nl); break;
      default: stage<T, INV, 7>(b0, b1, n, ns, nl); break;
    }
    ns *= R;
    __syncthreads();
    Cx<T>* t = b0;
    b0 = b1;
    b1 = t;
  }
  move_lines<T>(p, line0, nl, dst, b0, false);
}

// exact O(n^2) DFT of one LDS-resident line per workgroup (lengths with a prime factor > 7)
template <typename T, bool INV>
__global__ void __launch_bounds__(kFftThreads) fft_direct_kernel(FftPlan p, const Cx<T>* __restrict__ src,
                                                                 Cx<T>* dst) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  Cx<T>* x = reinterpret_cast<Cx<T>*>(smem_raw);
  const int n = (int)p.n;
  const int64_t line = blockIdx.x;
  move_lines<T>(p, line, 1, src, x, true);
  __syncthreads();
  Cx<T> out[8];
  int cnt = 0;
  for (int k = threadIdx.x; k < n; k += kFftThreads) {
    Cx<T> acc{T(0), T(0)};
    for (int j = 0; j < n; ++j) acc = cadd(acc, cmul(x[j], twiddle<T, INV>((int)(((int64_t)j * k) % n), n)));
    if (cnt < 8) out[cnt] = acc;
    ++cnt;
  }
  __syncthreads();  // every thread has read the whole line
  cnt = 0;
  for (int k = threadIdx.x; k < n; k += kFftThreads) x[k] = out[cnt++];
  __syncthreads();
  move_lines<T>(p, line, 1, dst, x, false);
}

bool factor(int64_t n, FftPlan& p) {
  p.nst = 0;
  for (int r : {8, 4, 2, 3, 5, 7}) {
    while (n % r == 0) {
      if (p.nst == kMaxStages) return false;
      p.radix[p.nst++] = r;
      n /= r;
    }
  }
  return n == 1;
}

template <typename T>
int fft_entry(int ndim, const int64_t* shape, int naxes, const int* axes, int64_t stack, int inverse, const void* in,
              void* out, hipStream_t st) {
  PXA_CHECK_ARG(ndim >= 1 && ndim <= 8 && shape && naxes >= 0 && naxes <= ndim && stack >= 0);
  PXA_CHECK_ARG(naxes == 0 || axes != nullptr);
  int64_t total = stack;
  for (int d = 0; d < ndim; ++d) {
    PXA_CHECK_ARG(shape[d] >= 1);
    total *= shape[d];
  }
  if (total == 0) return PXA_OK;
  PXA_CHECK_ARG(in && out);
  for (int i = 0; i < naxes; ++i) {
    PXA_CHECK_ARG(axes[i] >= 0 && axes[i] < ndim);
    for (int j = 0; j < i; ++j) PXA_CHECK_ARG(axes[i] != axes[j]);
  }
  const void* src = in;
  for (int i = 0; i < naxes; ++i) {
    const int a = axes[i];
    FftPlan p;
    p.n = shape[a];
    p.inner = 1;
    for (int d = a + 1; d < ndim; ++d) p.inner *= shape[d];
    p.lines = total / p.n;
    if (p.n == 1) continue;
    const size_t line_bytes = (size_t)p.n * sizeof(Cx<T>);
    const bool smooth = factor(p.n, p);
    if (smooth && 2 * line_bytes <= kFftLds) {
      int lpb = (int)(kFftLds / (2 * line_bytes));
      if (lpb > 16) lpb = 16;
      if (p.inner > 1 && lpb > p.inner) lpb = (int)p.inner;
      p.lpb = lpb;
      const int64_t blocks = (p.lines + lpb - 1) / lpb;
      PXA_CHECK_ARG(blocks <= 0x7fffffff);
      const size_t smem = 2 * (size_t)lpb * line_bytes;
      auto kern = inverse ? fft_stockham_kernel<T, true> : fft_stockham_kernel<T, false>;
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
      hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kFftThreads), smem, st, p, (const Cx<T>*)src,
                         (Cx<T>*)out);
    } else {
      if (line_bytes > kFftLds || p.n > 8 * kFftThreads) return PXA_ERR_UNSUPPORTED;
      PXA_CHECK_ARG(p.lines <= 0x7fffffff);
      p.lpb = 1;
      auto kern = inverse ? fft_direct_kernel<T, true> : fft_direct_kernel<T, false>;
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)line_bytes);
      hipLaunchKernelGGL(kern, dim3((unsigned)p.lines), dim3(kFftThreads), line_bytes, st, p, (const Cx<T>*)src,
                         (Cx<T>*)out);
    }
    const int e = last_launch_status();
    if (e) return e;
    src = out;
  }
  if (src == in && in != out)  // no axis transformed: plain copy
    return (int)hipMemcpyAsync(out, in, (size_t)total * sizeof(Cx<T>), hipMemcpyDeviceToDevice, st);
  return PXA_OK;
}

template <typename T>
__global__ void __launch_bounds__(kBlock) real_to_complex_kernel(int64_t n, const T* __restrict__ x,
                                                                 Cx<T>* __restrict__ z) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) z[i] = Cx<T>{x[i], T(0)};
}
template <typename T>
__global__ void __launch_bounds__(kBlock) complex_real_kernel(int64_t n, const Cx<T>* __restrict__ z,
                                                              T* __restrict__ x) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] = z[i].re;
}

// out[i] = a[i] * b[i % nb] (b conjugated if CONJ): spectrum product of an FFT convolution
template <typename T, bool CONJ>
__global__ void __launch_bounds__(kBlock) cmul_kernel(int64_t n, int64_t nb, const Cx<T>* __restrict__ a,
                                                      const Cx<T>* __restrict__ b, Cx<T>* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    Cx<T> w = b[i % nb];
    if (CONJ) w.im = -w.im;
    out[i] = cmul(a[i], w);
  }
}

}  // namespace
}  // namespace pxa

using namespace pxa;

extern "C" {

int pxa_fft(int dtype, int ndim, const int64_t* shape, int naxes, const int* axes, int64_t stack, int inverse,
            const void* in, void* out, void* stream) {
  PXA_DISPATCH(dtype, T, return fft_entry<T>(ndim, shape, naxes, axes, stack, inverse, in, out, as_stream(stream)));
}

int pxa_complex_mul(int dtype, int64_t n, int64_t nb, const void* a, const void* b, int conj_b, void* out,
                    void* stream) {
  PXA_CHECK_ARG(n >= 0 && nb >= 1);
  if (n == 0) return PXA_OK;
  PXA_CHECK_ARG(a && b && out);
  PXA_DISPATCH(dtype, T, {
    if (conj_b)
      hipLaunchKernelGGL((cmul_kernel<T, true>), dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), n, nb,
                         (const Cx<T>*)a, (const Cx<T>*)b, (Cx<T>*)out);
    else
      hipLaunchKernelGGL((cmul_kernel<T, false>), dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), n, nb,
                         (const Cx<T>*)a, (const Cx<T>*)b, (Cx<T>*)out);
    return last_launch_status();
  });
}

int pxa_real_to_complex(int dtype, int64_t n, const void* x, void* z, void* stream) {
  PXA_CHECK_ARG(n >= 0);
  if (n == 0) return PXA_OK;
  PXA_CHECK_ARG(x && z);
  PXA_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((real_to_complex_kernel<T>), dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), n,
                       (const T*)x, (Cx<T>*)z);
    return last_launch_status();
  });
}

int pxa_complex_real_part(int dtype, int64_t n, const void* z, void* x, void* stream) {
  PXA_CHECK_ARG(n >= 0);
  if (n == 0) return PXA_OK;
  PXA_CHECK_ARG(x && z);
  PXA_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((complex_real_kernel<T>), dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), n,
                       (const Cx<T>*)z, (T*)x);
    return last_launch_status();
  });
}

}  // extern "C"
