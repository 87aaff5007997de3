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
#include <cmath>
#include <map>
#include <mutex>
#include <set>
#include <utility>
#include <vector>

#include "common.hpp"

#ifndef PXA_PROBES
#define PXA_PROBES 0
#endif

namespace pxa {
namespace {

constexpr bool kFftProbes = PXA_PROBES != 0;
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
// fp32: complex arithmetic on 2-vectors, so that it issues as packed fp32 (v_pk_add / v_pk_mul / v_pk_fma:
// two lanes' worth of fp32 per instruction; the FFT kernels are VALU-bound at these counts)
typedef float PkF32 __attribute__((ext_vector_type(2)));
__device__ inline PkF32 pk(Cx<float> a) { return PkF32{a.re, a.im}; }
__device__ inline Cx<float> unpk(PkF32 a) { return Cx<float>{a.x, a.y}; }
template <>
__device__ inline Cx<float> cadd(Cx<float> a, Cx<float> b) {
  return unpk(pk(a) + pk(b));
}
template <>
__device__ inline Cx<float> csub(Cx<float> a, Cx<float> b) {
  return unpk(pk(a) - pk(b));
}
template <>
__device__ inline Cx<float> cmul(Cx<float> a, Cx<float> b) {
  // (ar br, ar bi), then + (-ai bi, ai br): the lane selects and the negation ride in the VOP3P modifiers
  // (written out: the compiler materialises the swapped operand with moves)
  PkF32 t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(pk(a)), "v"(pk(b)));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
      : "=v"(r) : "v"(pk(a)), "v"(pk(b)), "v"(t));
  return unpk(r);
}
// a + (-i) d (forward) / a + i d (inverse), and a - (-i) d / a - i d, in one packed add each
template <typename T, bool INV>
__device__ inline Cx<T> add_mi(Cx<T> a, Cx<T> d) {
  return cadd(a, mul_mi<T, INV>(d));
}
template <typename T, bool INV>
__device__ inline Cx<T> sub_mi(Cx<T> a, Cx<T> d) {
  return csub(a, mul_mi<T, INV>(d));
}
__device__ inline PkF32 pk_add_swap_neg_hi(PkF32 a, PkF32 d) {  // (a.re + d.im, a.im - d.re)
  PkF32 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(d));
  return r;
}
__device__ inline PkF32 pk_add_swap_neg_lo(PkF32 a, PkF32 d) {  // (a.re - d.im, a.im + d.re)
  PkF32 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(d));
  return r;
}
template <>
__device__ inline Cx<float> add_mi<float, false>(Cx<float> a, Cx<float> d) {
  return unpk(pk_add_swap_neg_hi(pk(a), pk(d)));
}
template <>
__device__ inline Cx<float> add_mi<float, true>(Cx<float> a, Cx<float> d) {
  return unpk(pk_add_swap_neg_lo(pk(a), pk(d)));
}
template <>
__device__ inline Cx<float> sub_mi<float, false>(Cx<float> a, Cx<float> d) {
  return unpk(pk_add_swap_neg_lo(pk(a), pk(d)));
}
template <>
__device__ inline Cx<float> sub_mi<float, true>(Cx<float> a, Cx<float> d) {
  return unpk(pk_add_swap_neg_hi(pk(a), pk(d)));
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
  const Cx<T> t2 = cadd(v[1], v[3]), d3 = csub(v[1], v[3]);
  v[0] = cadd(t0, t2);
  v[2] = csub(t0, t2);
  v[1] = add_mi<T, INV>(t1, d3);
  v[3] = sub_mi<T, INV>(t1, d3);
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
  const Cx<T> p1 = cmul(o[1], w1), p3 = cmul(o[3], w3);
  v[0] = cadd(e[0], o[0]);
  v[4] = csub(e[0], o[0]);
  v[1] = cadd(e[1], p1);
  v[5] = csub(e[1], p1);
  v[2] = add_mi<T, INV>(e[2], o[2]);
  v[6] = sub_mi<T, INV>(e[2], o[2]);
  v[3] = cadd(e[3], p3);
  v[7] = csub(e[3], p3);
}
// 16-point DFT as 4 x 4: DFTs of the stride-4 subsequences, twiddles W16^(n1 k2), DFTs across (fp32 LDS stages)
template <typename T, bool INV>
__device__ inline void dft16(Cx<T>* v) {
  Cx<T> a[4][4];
#pragma unroll
  for (int n1 = 0; n1 < 4; ++n1) {
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) a[n1][n2] = v[4 * n2 + n1];
    dft4<T, INV>(a[n1]);  // a[n1][k2] = sum_n2 x[4 n2 + n1] W4^(n2 k2)
  }
  const T c = T(0.92387953251128675613), sn = T(0.38268343236508977173), h = T(0.70710678118654752440);
  const T sg = INV ? T(1) : T(-1);
  // W16^m for m = n1 k2 in {1, 2, 3, 4, 6, 9}
  const Cx<T> w1{c, sg * sn}, w2{h, sg * h}, w3{sn, sg * c}, w6{-h, sg * h}, w9{-c, sg * -sn};
  a[1][1] = cmul(a[1][1], w1);
  a[1][2] = cmul(a[1][2], w2);
  a[1][3] = cmul(a[1][3], w3);
  a[2][1] = cmul(a[2][1], w2);
  a[2][2] = mul_mi<T, INV>(a[2][2]);
  a[2][3] = cmul(a[2][3], w6);
  a[3][1] = cmul(a[3][1], w3);
  a[3][2] = cmul(a[3][2], w6);
  a[3][3] = cmul(a[3][3], w9);
#pragma unroll
  for (int k2 = 0; k2 < 4; ++k2) {
    Cx<T> b[4] = {a[0][k2], a[1][k2], a[2][k2], a[3][k2]};
    dft4<T, INV>(b);  // X[k2 + 4 k1] = sum_n1 a[n1][k2] W4^(n1 k1)
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) v[k2 + 4 * k1] = b[k1];
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
  int pitch;                // fft_lds_kernel: LDS elements per line
  int no_fast;              // fft_lds_kernel: 1 = generic load / store paths only (PXA_TUNE_FFT_KERNEL bit 1024, A/B)
  int probe;                // fft_lds_kernel, probe build only: 16 skip stages, 32 skip loads, 64 skip stores, 128 no twiddle loads
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

// ---- in-place FFT of lines resident in LDS (PXA_TUNE_FFT_KERNEL 0, the default)
// The ping-pong kernel above keeps two copies of its lines (so only 2 lines of 2048 fp32 per workgroup:
// 16-B pieces of each row on a strided axis, 3.1x the compulsory HBM bytes, profiles/r04t_fft_pmc.txt),
// writes each Stockham stage with stride R (8-way LDS bank conflicts at R = 8: 6.7 M extra cycles against
// 2.8 M active) and evaluates a sincospi per butterfly.  This one: one copy of 64 or 128 KB of lines per
// workgroup (4 / 8 lines of 2048 fp32: 32- / 64-B pieces of each row on a strided axis, adjacent line groups
// on one XCD so that the rest of each 128-B line is an L2 hit), every stage in place -- all threads read their butterflies'
// inputs into registers, barrier, write the outputs -- on swizzled lines (fft_padi: no bank conflicts),
// twiddles w_n^m read from a table built once per length in double precision (exact to the rounding of T).
// Power-of-two lengths.

// TH threads per workgroup and TH * 128 bytes of line data: 512 threads / 64 KB (two workgroups per CU) or
// 1024 / 128 KB (one; twice the lines per workgroup, for strided axes and lines up to 16384 fp32)
template <typename T, int TH>
struct LdsFft {
  static constexpr int E = (int)(TH * 128 / sizeof(Cx<T>));  // elements per workgroup: 8192 / 16384 fp32
  static constexpr int PER = E / TH;                          // per thread and stage: 16 fp32, 8 fp64
};

// Position m of a line at m ^ ((m >> 3) & 15) (a permutation within aligned blocks of 16), lines at a pitch
// of n + 16 / min(L, 16): every Stockham stage's reads and writes and both load / store orders are free of
// bank conflicts for the power-of-two lengths (checked with the MI355X_MICROARCH.md bank model)
__host__ __device__ inline int fft_padi(int i) { return i ^ ((i >> 3) & 15); }
__host__ __device__ inline int fft_pitch(int n, int L) { return n + 16 / (L < 16 ? L : 16); }

// x / d and x % d for x, d < 2^16 by one multiply-high (m = floor((2^32 - 1) / d) + 1 is exact there)
struct FastDiv {
  unsigned d, m;
  __device__ explicit FastDiv(unsigned dd) : d(dd), m(0xFFFFFFFFu / dd + 1u) {}
  __device__ inline unsigned div(unsigned x) const { return d == 1u ? x : __umulhi(x, m); }
};

template <typename T, bool INV, int R>
__device__ inline void dft_r(Cx<T>* v) {
  if constexpr (R == 2) dft2<T, INV>(v);
  else if constexpr (R == 4) dft4<T, INV>(v);
  else if constexpr (R == 8) dft8<T, INV>(v);
  else if constexpr (R == 16) dft16<T, INV>(v);
  else dft_odd<T, INV, R>(v);
}

// One radix-R Stockham stage over L padded lines (pitch P) in place: v[r] = x[j + r n / R],
// twiddled by w_{ns R}^(r (j mod ns)) = tw[ns + (j mod ns)] ^ r, DFT_R, written to
// (j div ns) ns R + (j mod ns) + r ns.  n / R = 2^lnr and ns = 2^lns (power-of-two lengths): indices by
// shifts and masks.  A step that is a multiple of 128 leaves bits 0-6 alone, so fft_padi(x + r step) =
// fft_padi(x) + r step there: one address per butterfly (the reads for n >= 128 R, the writes of the
// stages with ns >= 128) instead of one swizzle per element.
template <typename T, bool INV, int R, int TH>
__device__ inline void lds_stage(Cx<T>* buf, int P, int lnr, int L, int lns, const Cx<T>* __restrict__ tw,
                                 bool probe_tw = false) {
  constexpr int NB = (LdsFft<T, TH>::PER + R - 1) / R;  // butterflies per thread
  const int nr = 1 << lnr, ns = 1 << lns;
  const int total = L << lnr;
  Cx<T> v[NB][R];
  Cx<T> w1[NB];  // w_{ns R}^k, loaded with the inputs: its latency overlaps the barrier
  auto read = [&](auto lin) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int t = (int)threadIdx.x + b * TH;
      if (t < total) {
        const int l = t >> lnr, j = t & (nr - 1);
        const Cx<T>* s = buf + l * P;
        if constexpr (lin()) {
          const Cx<T>* s0 = s + fft_padi(j);
#pragma unroll
          for (int r = 0; r < R; ++r) v[b][r] = s0[r * nr];
        } else {
#pragma unroll
          for (int r = 0; r < R; ++r) v[b][r] = s[fft_padi(j + r * nr)];
        }
        if (ns > 1) w1[b] = tw[ns + (j & (ns - 1))];  // consecutive k: coalesced
        if (kFftProbes && probe_tw) w1[b] = Cx<T>{T(1), T(0)};  // timing probe only (WRONG results)
      }
    }
  };
  if ((nr & 127) == 0) read(std::true_type{});
  else read(std::false_type{});
  __syncthreads();  // every input of the stage is in registers: the outputs may overwrite them
  auto write = [&](auto lin) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int t = (int)threadIdx.x + b * TH;
      if (t < total) {
        const int l = t >> lnr, j = t & (nr - 1);
        const int k = j & (ns - 1);
        if (ns > 1) {  // w^r: w^(2q) = (w^q)^2, w^(2q+1) = w^(2q) w -- a product chain of depth ~2 log2 r
          Cx<T> wp[R];
          wp[1] = w1[b];
          if (INV) wp[1].im = -wp[1].im;
#pragma unroll
          for (int r = 2; r < R; ++r) wp[r] = (r & 1) ? cmul(wp[r - 1], wp[1]) : cmul(wp[r / 2], wp[r / 2]);
#pragma unroll
          for (int r = 1; r < R; ++r) v[b][r] = cmul(v[b][r], wp[r]);
        }
        dft_r<T, INV, R>(v[b]);
        Cx<T>* d = buf + l * P;
        const int id = ((j - k) * R) + k;  // (j div ns) ns R + k
        if constexpr (lin()) {
          Cx<T>* d0 = d + fft_padi(id);
#pragma unroll
          for (int r = 0; r < R; ++r) d0[r << lns] = v[b][r];
        } else {
#pragma unroll
          for (int r = 0; r < R; ++r) d[fft_padi(id + (r << lns))] = v[b][r];
        }
      }
    }
  };
  if ((ns & 127) == 0) write(std::true_type{});
  else write(std::false_type{});
  __syncthreads();
}

// One complex element by a raw buffer access (voffset per thread, soffset uniform: no 64-bit address math)
typedef unsigned FftU2 __attribute__((ext_vector_type(2)));
typedef unsigned FftU4 __attribute__((ext_vector_type(4)));
template <typename T>
__device__ inline Cx<T> cx_buf_ld(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  if constexpr (sizeof(Cx<T>) == 8) return __builtin_bit_cast(Cx<T>, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
  else return __builtin_bit_cast(Cx<T>, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
template <typename T>
__device__ inline void cx_buf_st(Cx<T> v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  if constexpr (sizeof(Cx<T>) == 8) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(FftU2, v), r, voff, soff, 0);
  else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(FftU4, v), r, voff, soff, 0);
}

// XCD-aware group order (speed only): XCD g = blockIdx % 8 takes a contiguous band of line groups, so
// that the groups sharing the 128-B lines of a strided axis meet in one L2
__device__ inline unsigned fft_group(unsigned bid, unsigned nb) {
  const unsigned q8 = nb >> 3, r8 = nb & 7u, g8 = bid & 7u;
  return g8 * q8 + (g8 < r8 ? g8 : r8) + (bid >> 3);
}

// Power-of-two lengths (radices 8, 4, 2); the 3 / 5 / 7 butterflies held across the stage barrier would
// spill here (fp64 radix 7: 62 VGPRs), so lengths with an odd factor keep the ping-pong kernel.
template <typename T, bool INV, int TH>
__global__ void __launch_bounds__(TH, 4) fft_lds_kernel(FftPlan p, const Cx<T>* __restrict__ src, Cx<T>* dst,
                                                                 const Cx<T>* __restrict__ tw) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  Cx<T>* buf = reinterpret_cast<Cx<T>*>(smem_raw);
  const int n = (int)p.n;
  const int P = p.pitch;
  const int64_t line0 = (int64_t)fft_group(blockIdx.x, gridDim.x) * p.lpb;
  const int L = (int)((p.lines - line0) < p.lpb ? (p.lines - line0) : p.lpb);
  const int tot = L * n;
  const int lgn = 31 - __builtin_clz((unsigned)n);
  const FastDiv dl((unsigned)L);
  // load: contiguous axis position-fastest (each line one run), strided axis line-fastest (adjacent lines
  // adjacent in memory at each position); a thread's PER loads are all issued before the first LDS store.
  // Line-fastest with L dividing the thread count: the thread keeps one line, so its global base is
  // computed once (line_base / tstore_offset divide 64-bit integers)
  constexpr int PER = LdsFft<T, TH>::PER;
  const bool fixed_line = TH % L == 0;
  const int l_fix = (int)threadIdx.x % L, m_fix = (int)threadIdx.x / L, m_step = TH / L;
  auto coords = [&](int k, bool line_fast, int& l, int& m) {
    const int e = (int)threadIdx.x + k * TH;
    if (line_fast) {
      if (fixed_line) {
        l = l_fix;
        m = m_fix + k * m_step;
      } else {
        m = (int)dl.div((unsigned)e);
        l = e - m * L;
      }
    } else {
      l = e >> lgn;
      m = e & (n - 1);
    }
  };
  const bool lf_in = p.inner != 1;
  const bool lf_out = p.tn1 > 0 || p.inner != 1;
  // fixed line: element m at in_base + m * inner, out_base + m * out_step
  const int64_t in_base = lf_in && fixed_line ? line_base(line0 + l_fix, p.n, p.inner) : 0;
  const int64_t out_step = p.tn1 > 0 ? p.tn1 * p.inner : p.inner;
  const int64_t out_base = lf_out && fixed_line ? (p.tn1 > 0 ? tstore_offset(line0 + l_fix, 0, p)
                                                               : line_base(line0 + l_fix, p.n, p.inner))
                                                : 0;
  // global offset g and LDS slot sl of this thread's element k in the load (OUT false) or store order;
  // MODE 0 position-fastest, 1 line-fastest with a fixed line, 2 line-fastest (a template constant, so
  // that each load / store loop is free of branches and its values stay in registers)
  auto place = [&](int k, auto out, auto mode, int64_t& g, int& sl) {
    int l, m;
    coords(k, mode() != 0, l, m);
    sl = l * P + fft_padi(m);
    if constexpr (mode() == 0) g = (line0 + l) * n + m;
    else if constexpr (mode() == 1) g = out() ? out_base + (int64_t)m * out_step : in_base + (int64_t)m * p.inner;
    else if (out() && p.tn1 > 0) g = tstore_offset(line0 + l, m, p);
    else g = line_base(line0 + l, p.n, p.inner) + (int64_t)m * p.inner;
  };
  // full workgroups (tot == E) without the per-element bound
  auto load_lines = [&](auto full, auto mode) {
    T vr[PER], vi[PER];  // (a Cx<double> array here is left in scratch memory)
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (full() || (int)threadIdx.x + k * TH < tot) {
        int64_t g;
        int sl;
        place(k, std::false_type{}, mode, g, sl);
        const Cx<T> a = src[g];
        vr[k] = a.re;
        vi[k] = a.im;
      }
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (full() || (int)threadIdx.x + k * TH < tot) {
        int64_t g;
        int sl;
        place(k, std::false_type{}, mode, g, sl);
        buf[sl] = Cx<T>{vr[k], vi[k]};
      }
    }
  };
  auto store_lines = [&](auto full, auto mode) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (full() || (int)threadIdx.x + k * TH < tot) {
        int64_t g;
        int sl;
        place(k, std::true_type{}, mode, g, sl);
        dst[g] = buf[sl];
      }
    }
  };
  using M0 = std::integral_constant<int, 0>;
  using M1 = std::integral_constant<int, 1>;
  using M2 = std::integral_constant<int, 2>;
  const bool full = tot == LdsFft<T, TH>::E;
  auto dispatch = [&](bool lf, auto fn) {
    if (!lf) full ? fn(std::true_type{}, M0{}) : fn(std::false_type{}, M0{});
    else if (fixed_line) full ? fn(std::true_type{}, M1{}) : fn(std::false_type{}, M1{});
    else full ? fn(std::true_type{}, M2{}) : fn(std::false_type{}, M2{});
  };
  // Fast path (full groups; the contiguous axis, or line-fastest with the group's lines in one inner block,
  // the axis' span < 2 GB and no transposed store): element k of a thread at group base + voffset (per
  // thread) + k * sstep (uniform), its LDS slot at slot0 + a uniform step -- the generic path spends ~11
  // VALU per element on 64-bit offsets and swizzles
  const bool span_ok = p.n * p.inner * (int64_t)sizeof(Cx<T>) < ((int64_t)1 << 31);
  auto fast_ok = [&](bool lf, bool out) {
    return !p.no_fast && full && (!lf || (!(out && p.tn1 > 0) && fixed_line && p.inner % L == 0 && span_ok));
  };
  auto fast_lines = [&](auto out, auto lf, auto lin) {
    Cx<T>* gb;
    int voff, slot0, sstep;
    const int tid = (int)threadIdx.x;
    if constexpr (!lf()) {
      gb = (out() ? dst : const_cast<Cx<T>*>(src)) + line0 * n;
      voff = tid * (int)sizeof(Cx<T>);
      sstep = TH * (int)sizeof(Cx<T>);
      slot0 = (tid >> lgn) * P + fft_padi(tid & (n - 1));
    } else {
      gb = (out() ? dst : const_cast<Cx<T>*>(src)) + line_base(line0, p.n, p.inner);
      voff = (l_fix + m_fix * (int)p.inner) * (int)sizeof(Cx<T>);
      sstep = m_step * (int)p.inner * (int)sizeof(Cx<T>);
      slot0 = l_fix * P + fft_padi(m_fix);
    }
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(gb, (short)0, 0x7FFFFFFF, 0x00020000);
    auto slot = [&](int k) {
      if constexpr (!lf()) return slot0 + ((k * TH) >> lgn) * P + ((k * TH) & (n - 1));
      else if constexpr (lin()) return slot0 + k * m_step;  // m_step a multiple of 128: the swizzle is linear
      else return l_fix * P + fft_padi(m_fix + k * m_step);
    };
    if constexpr (!out()) {
      T vr[PER], vi[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const Cx<T> a = cx_buf_ld<T>(rs, voff, k * sstep);
        vr[k] = a.re;
        vi[k] = a.im;
      }
#pragma unroll
      for (int k = 0; k < PER; ++k) buf[slot(k)] = Cx<T>{vr[k], vi[k]};
    } else {
#pragma unroll
      // 16-B stores (fp64) take their whole offset in voffset, soffset = 0.  A buffer store of more than 8
      // bytes reads its data VGPRs after it issues; LLVM's hazard recognizer inserts the wait state before a
      // VALU write of those VGPRs only when soffset is not a register (GCNHazardRecognizer::createsVALUHazard),
      // but on gfx950 the hazard exists with an SGPR soffset too: the k-th store (soffset k * sstep in an SGPR)
      // was followed at once by `v_add_u32 v0, ...` (the next LDS address) into its data register v0, and now
      // and then the low dword of an fp64 result was that address (round-4 / r05b failure of
      // test_fft_vs_numpy[(2048, 2048)-(0, 1)-float64-True]: 16 values in one row, low dwords 0xd940..0xdc30,
      // high dwords exact; tests/test_gpu_fft.py::test_fft_f64_store_hazard_pattern).  8-B stores (fp32) have
      // no such hazard and keep the SGPR offset.
      for (int k = 0; k < PER; ++k) {
        if constexpr (sizeof(Cx<T>) > 8) cx_buf_st<T>(buf[slot(k)], rs, voff + k * sstep, 0);
        else cx_buf_st<T>(buf[slot(k)], rs, voff, k * sstep);
      }
    }
  };
  auto run_lines = [&](auto out, bool lf, auto generic) {
    if (!fast_ok(lf, out())) dispatch(lf, generic);
    else if (!lf) fast_lines(out, std::false_type{}, std::false_type{});
    else if ((m_step & 127) == 0) fast_lines(out, std::true_type{}, std::true_type{});
    else fast_lines(out, std::true_type{}, std::false_type{});
  };
  if (!(kFftProbes && (p.probe & 32))) run_lines(std::false_type{}, lf_in, load_lines);
  __syncthreads();
  int lns = 0;
  for (int s = 0; s < (kFftProbes && (p.probe & 16) ? 0 : p.nst); ++s) {
    const int R = p.radix[s];
    int lg = lgn;
    asm volatile("" : "+s"(lg));  // per stage: keeps the stages' thread-invariant LDS addresses out of registers
    const bool ptw = kFftProbes && (p.probe & 128);  // probe: no twiddle loads
    if (R == 16) {
      if constexpr (sizeof(T) == 4) lds_stage<T, INV, 16, TH>(buf, P, lg - 4, L, lns, tw, ptw);
    } else if (R == 8) lds_stage<T, INV, 8, TH>(buf, P, lg - 3, L, lns, tw, ptw);
    else if (R == 4) lds_stage<T, INV, 4, TH>(buf, P, lg - 2, L, lns, tw, ptw);
    else lds_stage<T, INV, 2, TH>(buf, P, lg - 1, L, lns, tw, ptw);
    lns += R == 16 ? 4 : R == 8 ? 3 : R == 4 ? 2 : 1;
  }
  if (kFftProbes && (p.probe & 64)) return;
  // store: the transposed four-step store and strided axes line-fastest, the contiguous axis position-fastest
  run_lines(std::true_type{}, lf_out, store_lines);
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

// Radices of the in-LDS kernel (powers of two): 16 first for fp32 (16 values per thread: one radix-16
// butterfly, three LDS round trips instead of four at 2048), 8 for fp64 (8 per thread); then 8 / 4 / 2
template <typename T>
bool factor_lds(int64_t n, FftPlan& p) {
  p.nst = 0;
  for (int r : {sizeof(T) == 4 ? 16 : 8, 8, 4, 2}) {
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

// Twiddle tables of the power-of-two in-LDS kernel, in static device memory of the code object (no allocation at
// run time): the table of length n occupies [n, 2n) of g_tw_f32 / g_tw_f64 (n <= LdsFft<T, 1024>::E: 16384 fp32,
// 8192 fp64; 256 KB each).  The first call for a length (per device) enqueues tw_fill_kernel on the caller's
// stream and marks the table built; calls during a stream capture enqueue the fill into the graph every time and
// mark nothing (the graph may never run), so pxa_fft_ex is graph-capturable on a length never seen before
// (tests/test_gpu_fft.py::test_fft_graph_capture_cold_length).  No allocation, no synchronisation: a concurrent
// first use of one length on a second stream must be ordered after the first by the caller, as for any buffer.
constexpr int kTwMaxF32 = 16384, kTwMaxF64 = 8192;
__device__ Cx<float> g_tw_f32[2 * kTwMaxF32];
__device__ Cx<double> g_tw_f64[2 * kTwMaxF64];

template <typename T>
constexpr int tw_max() {
  return sizeof(T) == 4 ? kTwMaxF32 : kTwMaxF64;
}
template <typename T>
__device__ inline Cx<T>* tw_store();
template <>
__device__ inline Cx<float>* tw_store<float>() {
  return g_tw_f32;
}
template <>
__device__ inline Cx<double>* tw_store<double>() {
  return g_tw_f64;
}

// Stage twiddles: the stage of span ns and radix R reads w_{ns R}^k, k < ns, at tw[ns + k] (the spans are
// distinct powers of two, so the ranges [ns, 2 ns) do not overlap; n entries in all, the rest 1 + 0i).
// exp(-2 pi i k / (ns R)) from sincospi of the exact dyadic argument 2k / (ns R) in double, rounded to T
// (fp32: correctly rounded but for results within an fp64 ulp of a rounding boundary; fp64: ~1 ulp).
template <typename T>
__global__ void __launch_bounds__(256) tw_fill_kernel(FftPlan p) {
  const int64_t n = p.n;
  Cx<T>* tw = tw_store<T>() + n;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    Cx<T> w{T(1), T(0)};
    int64_t ns = 1;
    for (int s = 0; s < p.nst; ++s) {
      const int R = p.radix[s];
      if (ns > 1 && j >= ns && j < 2 * ns) {
        double sn, cs;
        sincospi(2.0 * (double)(j - ns) / (double)(ns * R), &sn, &cs);
        w = Cx<T>{(T)cs, (T)(-sn)};
      }
      ns *= R;
    }
    tw[j] = w;
  }
}

template <typename T>
const Cx<T>* twiddle_table(const FftPlan& p, hipStream_t st) {
  if (p.n > tw_max<T>()) return nullptr;
  static std::mutex mu;
  static std::map<int, Cx<T>*> bases;       // device address of the table store, per device
  static std::set<std::pair<int, int64_t>> built;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  auto bi = bases.find(dev);
  if (bi == bases.end()) {
    void* a = nullptr;
    const hipError_t e = sizeof(T) == 4 ? hipGetSymbolAddress(&a, HIP_SYMBOL(g_tw_f32))
                                        : hipGetSymbolAddress(&a, HIP_SYMBOL(g_tw_f64));
    if (e != hipSuccess || a == nullptr) return nullptr;
    bi = bases.emplace(dev, (Cx<T>*)a).first;
  }
  const std::pair<int, int64_t> key{dev, p.n};
  if (!built.count(key)) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cap) != hipSuccess) return nullptr;
    const unsigned blocks = (unsigned)((p.n + 255) / 256);
    hipLaunchKernelGGL(tw_fill_kernel<T>, dim3(blocks), dim3(256), 0, st, p);
    if (hipGetLastError() != hipSuccess) return nullptr;
    if (cap == hipStreamCaptureStatusNone) built.insert(key);
  }
  return bi->second + p.n;
}

template <typename T>
bool lds_fft_fits(int64_t n) {  // powers of two (see fft_lds_kernel)
  return n >= 2 && n <= LdsFft<T, 1024>::E && (n & (n - 1)) == 0 &&
         (size_t)fft_pitch((int)n, 1) * sizeof(Cx<T>) <= kFftLdsMax;
}

// Workgroup size: 1024 threads / 128 KB for lines longer than 64 KB, and on strided axes whose 512-thread
// group would hold only 1 or 2 lines (8- or 16-B row pieces: 4096^2 fp32 axis 0 170 -> 122 us); 512 / 64 KB
// otherwise (2048^2 axis 0: equal, 23.0 vs 23.3 us; 256^3 axes 0 / 1: 82 / 74 us against 96 / 80 with 1024,
// profiles/r04zf_fft_th.txt).  PXA_TUNE_FFT_KERNEL bit 256 forces 512, bit 512 forces 1024 (A/B).
template <typename T>
int lds_fft_threads(const FftPlan& p) {
  const int64_t t = tuning(PXA_TUNE_FFT_KERNEL);
  if (p.n > LdsFft<T, 512>::E || (t & 512)) return 1024;
  if (t & 256) return 512;
  return p.inner > 1 && 2 * p.n >= LdsFft<T, 512>::E ? 1024 : 512;
}

template <typename T, int TH>
int launch_lds_fft_th(FftPlan p, bool inv, const Cx<T>* src, Cx<T>* dst, const Cx<T>* tw, hipStream_t st) {
  int L = (int)(LdsFft<T, TH>::E / p.n);
  if (L > p.lines) L = (int)p.lines;
  if (p.inner > 1 && L > p.inner) L = (int)p.inner;
  if (L < 1) L = 1;
  while (L > 1 && (size_t)L * fft_pitch((int)p.n, L) * sizeof(Cx<T>) > kFftLdsMax) L /= 2;  // short lines: pitch pad
  p.lpb = L;
  p.pitch = fft_pitch((int)p.n, L);
  p.probe = kFftProbes ? (tuning(PXA_TUNE_FFT_KERNEL) & 0xF0) : 0;
  p.no_fast = (tuning(PXA_TUNE_FFT_KERNEL) & 1024) ? 1 : 0;
  const int64_t blocks = (p.lines + L - 1) / L;
  PXA_CHECK_ARG(blocks <= 0x7fffffff);
  const size_t smem = (size_t)L * p.pitch * sizeof(Cx<T>);
  if (smem > kFftLdsMax) return PXA_ERR_UNSUPPORTED;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fft_lds_kernel<T, false, TH>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kFftLdsMax);
    (void)hipFuncSetAttribute((const void*)fft_lds_kernel<T, true, TH>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kFftLdsMax);
    attr = true;
  }
  auto kern = inv ? fft_lds_kernel<T, true, TH> : fft_lds_kernel<T, false, TH>;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(TH), smem, st, p, src, dst, tw);
  return last_launch_status();
}

template <typename T>
int launch_lds_fft(FftPlan p, bool inv, const Cx<T>* src, Cx<T>* dst, hipStream_t st) {
  if (!factor_lds<T>(p.n, p)) return PXA_ERR_UNSUPPORTED;
  const Cx<T>* tw = twiddle_table<T>(p, st);
  if (tw == nullptr) return launch_stockham<T>(p, inv, src, dst, st);  // (no table for this length)
  return lds_fft_threads<T>(p) == 1024 ? launch_lds_fft_th<T, 1024>(p, inv, src, dst, tw, st)
                                       : launch_lds_fft_th<T, 512>(p, inv, src, dst, tw, st);
}

// the in-LDS transform of one axis: the in-place kernel (default) or the ping-pong kernel (A/B)
template <typename T>
int launch_lines(FftPlan p, bool inv, const Cx<T>* src, Cx<T>* dst, hipStream_t st) {
  if ((tuning(PXA_TUNE_FFT_KERNEL) & 15) == 0 && lds_fft_fits<T>(p.n)) return launch_lds_fft<T>(p, inv, src, dst, st);
  return launch_stockham<T>(p, inv, src, dst, st);
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
  if (stockham_fits<T>(n)) return launch_lines<T>(p, inv, src, dst, st);
  // power-of-two lines up to 128 KB: one in-LDS pass instead of the four-step's three (its workspace, sized
  // by axis_work regardless of the tuning knob, is then unused)
  if ((tuning(PXA_TUNE_FFT_KERNEL) & 15) == 0 && lds_fft_fits<T>(n)) return launch_lines<T>(p, inv, src, dst, st);
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
    int e = launch_lines<T>(p1, inv, src, dst, st);
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
    e = launch_lines<T>(p2, inv, dst, work, st);
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
