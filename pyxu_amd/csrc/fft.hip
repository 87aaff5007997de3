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
// Lines longer than LDS holds: smooth lengths by the four-step split n = n1 n2 (n1-point DFTs along
// the stride-n2 axis, twiddles w_n^(k1 j2), n2-point DFTs stored transposed into a workspace, copied
// back); other lengths by Bluestein's chirp-z (chirp, 2^k-point FFT convolution with the chirp filter,
// chirp), so every length runs, as in the reference's scipy.fft.
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
  int64_t tn1;              // 0: results back in place of the line; > 0: four-step transposed store (below)
  int lpb;                  // lines per workgroup
  int nst;
  int radix[kMaxStages];
};

// Four-step transposed store: the line (o, k1, i) of an (outer, tn1, n, inner) view writes its element
// k2 to (o, k2, k1, i) of the (outer, n, tn1, inner) view, i.e. offset (o n tn1 + k2 tn1 + k1) inner + i.
__device__ inline int64_t tstore_offset(int64_t line, int64_t m, const FftPlan& p) {
  const int64_t per = p.tn1 * p.inner;
  const int64_t o = line / per, rem = line - o * per;
  const int64_t k1 = rem / p.inner, i = rem - k1 * p.inner;
  return (o * p.n * p.tn1 + m * p.tn1 + k1) * p.inner + i;
}

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
  if (!to_lds && p.tn1 > 0) {  // transposed store: adjacent lines land in adjacent elements
    for (int i = threadIdx.x; i < nl * n; i += kFftThreads) {
      const int m = i / nl, l = i - m * nl;
      const_cast<Cx<T>*>(g)[tstore_offset(line0 + l, m, p)] = lds[l * n + m];
    }
    return;
  }
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

bool smooth(int64_t n) {
  for (int r : {2, 3, 5, 7})
    while (n % r == 0) n /= r;
  return n == 1;
}

// One workgroup may take the whole LDS for a single long line; several lines per workgroup share 64 KB
// (two workgroups per CU).
constexpr size_t kFftLdsMax = 160 * 1024;
constexpr int64_t kDirectMaxN = 8 * kFftThreads;

template <typename T>
bool stockham_fits(int64_t n) {
  return smooth(n) && 2 * (size_t)n * sizeof(Cx<T>) <= kFftLdsMax;
}
template <typename T>
bool direct_fits(int64_t n) {
  return n <= kDirectMaxN && (size_t)n * sizeof(Cx<T>) <= kFftLdsMax;
}
// four-step split n = n1 n2 with both factors Stockham-resident, n1 the largest such divisor <= sqrt(n)
template <typename T>
int64_t four_step_n1(int64_t n) {
  if (!smooth(n)) return 0;
  for (int64_t n1 = (int64_t)sqrt((double)n) + 1; n1 >= 2; --n1)
    if (n % n1 == 0 && n1 * n1 <= n && stockham_fits<T>(n1) && stockham_fits<T>(n / n1)) return n1;
  return 0;
}
int64_t next_pow2(int64_t v) {
  int64_t m = 1;
  while (m < v) m <<= 1;
  return m;
}

// Workspace (complex elements) of one axis transform of `lines` lines of length n; -1: unsupported.
template <typename T>
int64_t axis_work(int64_t n, int64_t lines) {
  if (n == 1 || stockham_fits<T>(n) || (!smooth(n) && direct_fits<T>(n))) return 0;
  if (smooth(n)) return four_step_n1<T>(n) ? n * lines : -1;
  const int64_t m = next_pow2(2 * n - 1);  // Bluestein: a (lines x m), b (m), then the FFT_m's own
  const int64_t inner = axis_work<T>(m, lines);
  return inner < 0 ? -1 : lines * m + m + inner;
}

template <typename T>
int launch_stockham(FftPlan p, bool inv, const Cx<T>* src, Cx<T>* dst, hipStream_t st) {
  if (!factor(p.n, p)) return PXA_ERR_UNSUPPORTED;
  const size_t line_bytes = (size_t)p.n * sizeof(Cx<T>);
  int lpb = (int)(kFftLds / (2 * line_bytes));
  if (lpb > 16) lpb = 16;
  if (lpb < 1) lpb = 1;
  if (p.inner > 1 && lpb > p.inner) lpb = (int)p.inner;
  p.lpb = lpb;
  const int64_t blocks = (p.lines + lpb - 1) / lpb;
  PXA_CHECK_ARG(blocks <= 0x7fffffff);
  const size_t smem = 2 * (size_t)lpb * line_bytes;
  if (smem > kFftLdsMax) return PXA_ERR_UNSUPPORTED;
  static bool attr = false;  // the dynamic-LDS ceiling is a property of the kernel: set once
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fft_stockham_kernel<T, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kFftLdsMax);
    (void)hipFuncSetAttribute((const void*)fft_stockham_kernel<T, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kFftLdsMax);
    attr = true;
  }
  auto kern = inv ? fft_stockham_kernel<T, true> : fft_stockham_kernel<T, false>;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kFftThreads), smem, st, p, src, dst);
  return last_launch_status();
}

template <typename T>
int launch_direct(FftPlan p, bool inv, const Cx<T>* src, Cx<T>* dst, hipStream_t st) {
  PXA_CHECK_ARG(p.lines <= 0x7fffffff);
  p.lpb = 1;
  const size_t line_bytes = (size_t)p.n * sizeof(Cx<T>);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fft_direct_kernel<T, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kFftLdsMax);
    (void)hipFuncSetAttribute((const void*)fft_direct_kernel<T, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kFftLdsMax);
    attr = true;
  }
  auto kern = inv ? fft_direct_kernel<T, true> : fft_direct_kernel<T, false>;
  hipLaunchKernelGGL(kern, dim3((unsigned)p.lines), dim3(kFftThreads), line_bytes, st, p, src, dst);
  return last_launch_status();
}

// four-step twiddle: element (o, k1, j2, i) of the (outer, n1, n2, inner) view times w_n^(k1 j2)
template <typename T, bool INV>
__global__ void __launch_bounds__(kBlock) four_step_twiddle_kernel(int64_t total, int64_t n1, int64_t n2,
                                                                   int64_t inner, Cx<T>* __restrict__ z) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n = n1 * n2;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    int64_t t = e / inner;
    const int64_t j2 = t % n2;
    t /= n2;
    const int64_t k1 = t % n1;
    const int64_t q = (k1 * j2) % n;
    if (q != 0) {
      T sn, c;
      sc_pi((T)(2 * q) / (T)n, &sn, &c);
      z[e] = cmul(z[e], Cx<T>{c, INV ? sn : -sn});
    }
  }
}

// Bluestein chirp w(j) = exp(-+ i pi j^2 / n) (exact rational phase: j^2 mod 2n)
template <typename T, bool INV>
__device__ inline Cx<T> chirp(int64_t j, int64_t n) {
  const int64_t q = (j * j) % (2 * n);
  T sn, c;
  sc_pi((T)q / (T)n, &sn, &c);
  return Cx<T>{c, INV ? sn : -sn};
}

// a[l][j] = src(l, j) w(j) for j < n, 0 for n <= j < m (lines gathered from any axis stride)
template <typename T, bool INV>
__global__ void __launch_bounds__(kBlock) bluestein_in_kernel(int64_t lines, int64_t n, int64_t inner, int64_t m,
                                                              const Cx<T>* __restrict__ src, Cx<T>* __restrict__ a) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < lines * m; e += stride) {
    const int64_t l = e / m, j = e - l * m;
    a[e] = j < n ? cmul(src[line_base(l, n, inner) + j * inner], chirp<T, INV>(j, n)) : Cx<T>{T(0), T(0)};
  }
}

// b[j] = conj w(d), d = j (j < n) or m - j (j > m - n), else 0: the circular chirp filter
template <typename T, bool INV>
__global__ void __launch_bounds__(kBlock) bluestein_filter_kernel(int64_t n, int64_t m, Cx<T>* __restrict__ b) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
    const int64_t d = j < n ? j : (j > m - n ? m - j : -1);
    b[j] = d < 0 ? Cx<T>{T(0), T(0)} : chirp<T, !INV>(d, n);
  }
}

// dst(l, k) = a[l][k] w(k) / m
template <typename T, bool INV>
__global__ void __launch_bounds__(kBlock) bluestein_out_kernel(int64_t lines, int64_t n, int64_t inner, int64_t m,
                                                               const Cx<T>* __restrict__ a, Cx<T>* dst) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const T inv_m = T(1) / (T)m;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < lines * n; e += stride) {
    const int64_t l = e / n, k = e - l * n;
    const Cx<T> v = cmul(a[l * m + k], chirp<T, INV>(k, n));
    dst[line_base(l, n, inner) + k * inner] = Cx<T>{v.re * inv_m, v.im * inv_m};
  }
}

// DFT of `lines` lines of length n and element stride `inner` (line l at line_base(l, n, inner)),
// src -> dst (may alias).  work: axis_work<T>(n, lines) complex elements.
template <typename T>
int fft_axis(int64_t n, int64_t inner, int64_t lines, bool inv, const Cx<T>* src, Cx<T>* dst, Cx<T>* work,
             hipStream_t st) {
  FftPlan p;
  p.n = n;
  p.inner = inner;
  p.lines = lines;
  p.tn1 = 0;
  if (stockham_fits<T>(n)) return launch_stockham<T>(p, inv, src, dst, st);
  if (!smooth(n) && direct_fits<T>(n)) return launch_direct<T>(p, inv, src, dst, st);
  if (axis_work<T>(n, lines) < 0) return PXA_ERR_UNSUPPORTED;
  if (work == nullptr) return PXA_ERR_ARG;
  const int64_t total = n * lines;
  if (smooth(n)) {  // four-step: n1-point DFTs, twiddles, n2-point DFTs stored transposed, copy back
    const int64_t n1 = four_step_n1<T>(n), n2 = n / n1;
    FftPlan p1 = p;
    p1.n = n1;
    p1.inner = n2 * inner;
    p1.lines = total / n1;
    int e = launch_stockham<T>(p1, inv, src, dst, st);
    if (e) return e;
    if (inv)
      hipLaunchKernelGGL((four_step_twiddle_kernel<T, true>), dim3(grid_for(total)), dim3(kBlock), 0, st, total, n1,
                         n2, inner, dst);
    else
      hipLaunchKernelGGL((four_step_twiddle_kernel<T, false>), dim3(grid_for(total)), dim3(kBlock), 0, st, total, n1,
                         n2, inner, dst);
    e = last_launch_status();
    if (e) return e;
    FftPlan p2 = p;
    p2.n = n2;
    p2.inner = inner;
    p2.lines = total / n2;
    p2.tn1 = n1;
    e = launch_stockham<T>(p2, inv, dst, work, st);
    if (e) return e;
    return (int)hipMemcpyAsync(dst, work, (size_t)total * sizeof(Cx<T>), hipMemcpyDeviceToDevice, st);
  }
  // Bluestein: chirp, m-point FFT convolution with the chirp filter (m = 2^k >= 2n - 1), chirp
  const int64_t m = next_pow2(2 * n - 1);
  Cx<T>* a = work;
  Cx<T>* b = a + lines * m;
  Cx<T>* w2 = b + m;
  if (inv) {
    hipLaunchKernelGGL((bluestein_in_kernel<T, true>), dim3(grid_for(lines * m)), dim3(kBlock), 0, st, lines, n,
                       inner, m, src, a);
    hipLaunchKernelGGL((bluestein_filter_kernel<T, true>), dim3(grid_for(m)), dim3(kBlock), 0, st, n, m, b);
  } else {
    hipLaunchKernelGGL((bluestein_in_kernel<T, false>), dim3(grid_for(lines * m)), dim3(kBlock), 0, st, lines, n,
                       inner, m, src, a);
    hipLaunchKernelGGL((bluestein_filter_kernel<T, false>), dim3(grid_for(m)), dim3(kBlock), 0, st, n, m, b);
  }
  int e = last_launch_status();
  if (e) return e;
  if ((e = fft_axis<T>(m, 1, lines, false, a, a, w2, st))) return e;
  if ((e = fft_axis<T>(m, 1, 1, false, b, b, w2, st))) return e;
  hipLaunchKernelGGL((cmul_kernel<T, false>), dim3(grid_for(lines * m)), dim3(kBlock), 0, st, lines * m, m, a, b, a);
  if ((e = last_launch_status())) return e;
  if ((e = fft_axis<T>(m, 1, lines, true, a, a, w2, st))) return e;
  if (inv)
    hipLaunchKernelGGL((bluestein_out_kernel<T, true>), dim3(grid_for(lines * n)), dim3(kBlock), 0, st, lines, n, inner,
                       m, a, dst);
  else
    hipLaunchKernelGGL((bluestein_out_kernel<T, false>), dim3(grid_for(lines * n)), dim3(kBlock), 0, st, lines, n,
                       inner, m, a, dst);
  return last_launch_status();
}

template <typename T>
int fft_check(int ndim, const int64_t* shape, int naxes, const int* axes, int64_t stack, int64_t& total) {
  PXA_CHECK_ARG(ndim >= 1 && ndim <= 8 && shape && naxes >= 0 && naxes <= ndim && stack >= 0);
  PXA_CHECK_ARG(naxes == 0 || axes != nullptr);
  total = stack;
  for (int d = 0; d < ndim; ++d) {
    PXA_CHECK_ARG(shape[d] >= 1);
    total *= shape[d];
  }
  for (int i = 0; i < naxes; ++i) {
    PXA_CHECK_ARG(axes[i] >= 0 && axes[i] < ndim);
    for (int j = 0; j < i; ++j) PXA_CHECK_ARG(axes[i] != axes[j]);
  }
  return PXA_OK;
}

// complex elements of workspace for the whole transform (max over the axes); -1: unsupported
template <typename T>
int64_t fft_work_elems(int ndim, const int64_t* shape, int naxes, const int* axes, int64_t stack) {
  int64_t total = 0;
  if (fft_check<T>(ndim, shape, naxes, axes, stack, total) != PXA_OK) return -1;
  int64_t need = 0;
  for (int i = 0; i < naxes && total > 0; ++i) {
    const int64_t n = shape[axes[i]];
    const int64_t w = axis_work<T>(n, total / n);
    if (w < 0) return -1;
    need = w > need ? w : need;
  }
  return need;
}

template <typename T>
int fft_entry(int ndim, const int64_t* shape, int naxes, const int* axes, int64_t stack, int inverse, const void* in,
              void* out, void* work, hipStream_t st) {
  int64_t total = 0;
  const int c = fft_check<T>(ndim, shape, naxes, axes, stack, total);
  if (c != PXA_OK) return c;
  if (total == 0) return PXA_OK;
  PXA_CHECK_ARG(in && out);
  const void* src = in;
  for (int i = 0; i < naxes; ++i) {
    const int a = axes[i];
    const int64_t n = shape[a];
    if (n == 1) continue;
    int64_t inner = 1;
    for (int d = a + 1; d < ndim; ++d) inner *= shape[d];
    const int64_t w = axis_work<T>(n, total / n);
    if (w < 0) return PXA_ERR_UNSUPPORTED;
    if (w > 0 && work == nullptr) return PXA_ERR_UNSUPPORTED;  // pxa_fft: no workspace given
    const int e = fft_axis<T>(n, inner, total / n, inverse != 0, (const Cx<T>*)src, (Cx<T>*)out, (Cx<T>*)work, st);
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

}  // namespace
}  // namespace pxa

using namespace pxa;

extern "C" {

int pxa_fft(int dtype, int ndim, const int64_t* shape, int naxes, const int* axes, int64_t stack, int inverse,
            const void* in, void* out, void* stream) {
  PXA_DISPATCH(dtype, T,
               return fft_entry<T>(ndim, shape, naxes, axes, stack, inverse, in, out, nullptr, as_stream(stream)));
}

size_t pxa_fft_workspace_bytes(int dtype, int ndim, const int64_t* shape, int naxes, const int* axes, int64_t stack) {
  int64_t e = -1;
  if (dtype == PXA_F32) e = fft_work_elems<float>(ndim, shape, naxes, axes, stack);
  else if (dtype == PXA_F64) e = fft_work_elems<double>(ndim, shape, naxes, axes, stack);
  if (e < 0) return (size_t)-1;
  return (size_t)e * (dtype == PXA_F32 ? sizeof(Cx<float>) : sizeof(Cx<double>));
}

int pxa_fft_ex(int dtype, int ndim, const int64_t* shape, int naxes, const int* axes, int64_t stack, int inverse,
               const void* in, void* out, void* work, void* stream) {
  PXA_DISPATCH(dtype, T,
               return fft_entry<T>(ndim, shape, naxes, axes, stack, inverse, in, out, work, as_stream(stream)));
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
