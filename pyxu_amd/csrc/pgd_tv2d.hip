// Fused PGD step for 2-D TV-regularised deblurring: one launch per solver iteration.
//
//   yk     = x + a (x - x_prev)
//   r      = H yk - y                                  (H: separable zero-boundary correlation)
//   q_d    = lam * (v_d - prox_{mu L21}(v)_d) / mu,     v = Grad yk (forward differences)
//   x_new  = prox_{tau G}( yk - tau (H^T r + Grad^T q) )
//
// Reference dataflow: PGD.m_step (opt/solver/pgd.py:173-191) through AddRule.grad,
// ChainRule.grad, ScaleRule.grad, ArgShiftRule.grad (abc/arithmetic.py), Stencil.apply/adjoint
// (operator/linop/stencil/stencil.py:441-461), Gradient (operator/linop/diff.py:1113-1265),
// moreau_envelope grad (abc/operator.py:1053-1058), L21Norm.prox (operator/func/norm.py:352-364),
// PositiveOrthant.prox / L1Norm.prox.
//
// One workgroup owns a TY x TX output tile and recomputes its halo: yk on (TY+4R) x (TX+4R),
// r on (TY+2R) x (TX+2R), q on (TY+1) x (TX+1), all staged in LDS.  HBM traffic per iteration
// is the compulsory 3 reads (x, x_prev, y) + 1 write (x_new) per pixel; halo re-reads hit L2.
// Each separable pass keeps a sliding window of taps in registers (one LDS read per input
// element per strip instead of one per tap).  Tiles are dealt so that each XCD works on a
// contiguous band of the image (vertical neighbours share that XCD's L2).
#include "common.hpp"

namespace pxa {
namespace {

constexpr int TY = 32;
constexpr int TX = 64;
constexpr int kThreads = 256;
constexpr int kMaxR = 8;

__host__ __device__ constexpr int odd_pitch(int w) { return w | 1; }
__host__ __device__ constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }

template <typename T>
struct PgdParams {
  int64_t stack, n0, n1;
  int64_t y_images;  // y is shared by stack entries s with equal s % y_images
  int tiles0, tiles1;
  int64_t ntiles;  // stack * tiles0 * tiles1
  T k0[2 * kMaxR + 1], k1[2 * kMaxR + 1];  // H taps, dense window offsets -R..R (code-gen order)
  T g0a, g0b, g1a, g1b;                     // forward-difference taps per axis (-1/h, 1/h)
  T lam, mu, a, tau, pw;
};

template <int R>
struct Layout {
  static constexpr int AR = TY + 4 * R, AC = TX + 4 * R, AP = odd_pitch(AC);  // yk (later r)
  static constexpr int P1R = TY + 2 * R, P1C = TX + 4 * R, P1P = odd_pitch(P1C);
  static constexpr int RR = TY + 2 * R, RC = TX + 2 * R;                        // r lives in A (pitch AP)
  static constexpr int P3R = TY, P3C = TX + 2 * R, P3P = odd_pitch(P3C);        // in B
  static constexpr int QR = TY + 1, QC = TX + 1, QP = odd_pitch(QC);            // q (2 comps) in B
  static constexpr int A_ELEMS = AR * AP;
  static constexpr int B_ELEMS_P1 = P1R * P1P;
  static constexpr int B_ELEMS_Q = 2 * QR * QP;
  static constexpr int B_ELEMS_P3 = P3R * P3P;
  static constexpr int B_ELEMS = B_ELEMS_P1 > B_ELEMS_Q ? (B_ELEMS_P1 > B_ELEMS_P3 ? B_ELEMS_P1 : B_ELEMS_P3)
                                                        : (B_ELEMS_Q > B_ELEMS_P3 ? B_ELEMS_Q : B_ELEMS_P3);
  // strip lengths (register windows) per pass, sized so one pass is ~one round of 256 threads
  static constexpr int NSEG_A = kThreads / P1C > 0 ? kThreads / P1C : 1;
  static constexpr int SEG_A = cdiv(P1R, NSEG_A);
  static constexpr int NSEG_B = kThreads / RR > 0 ? kThreads / RR : 1;
  static constexpr int SEG_B = cdiv(RC, NSEG_B);
  static constexpr int NSEG_C = kThreads / P3C > 0 ? kThreads / P3C : 1;
  static constexpr int SEG_C = cdiv(P3R, NSEG_C);
  static constexpr int NSEG_D = kThreads / TY;  // = 8
  static constexpr int SEG_D = TX / NSEG_D;     // = 8
};

// Vertical (axis-0) pass: dst[r][c] = sum_j k[j] src[r + j][c], r < nr, c < nc.
template <typename T, int R, int SEG>
__device__ inline void vpass(const T* __restrict__ src, int ps, T* __restrict__ dst, int pd, int nr, int nc,
                             const T* __restrict__ k) {
  const int nseg = cdiv(nr, SEG);
  for (int item = threadIdx.x; item < nc * nseg; item += kThreads) {
    const int c = item % nc, r0 = (item / nc) * SEG;
    T win[SEG + 2 * R];
#pragma unroll
    for (int j = 0; j < SEG + 2 * R; ++j) win[j] = (r0 + j < nr + 2 * R) ? src[(r0 + j) * ps + c] : T(0);
#pragma unroll
    for (int i = 0; i < SEG; ++i) {
      T acc = T(0);
#pragma unroll
      for (int j = 0; j <= 2 * R; ++j) acc += k[j] * win[i + j];
      if (r0 + i < nr) dst[(r0 + i) * pd + c] = acc;
    }
  }
}

// Horizontal (axis-1) pass: dst[r][c] = sum_j k[j] src[r][c + j].
template <typename T, int R, int SEG>
__device__ inline void hpass(const T* __restrict__ src, int ps, T* __restrict__ dst, int pd, int nr, int nc,
                             const T* __restrict__ k) {
  const int nseg = cdiv(nc, SEG);
  for (int item = threadIdx.x; item < nr * nseg; item += kThreads) {
    const int r = item / nseg, c0 = (item % nseg) * SEG;
    T win[SEG + 2 * R];
#pragma unroll
    for (int j = 0; j < SEG + 2 * R; ++j) win[j] = (c0 + j < nc + 2 * R) ? src[r * ps + c0 + j] : T(0);
#pragma unroll
    for (int i = 0; i < SEG; ++i) {
      T acc = T(0);
#pragma unroll
      for (int j = 0; j <= 2 * R; ++j) acc += k[j] * win[i + j];
      if (c0 + i < nc) dst[r * pd + c0 + i] = acc;
    }
  }
}

template <typename T>
__device__ inline T fast_recip(T v) {
  return T(1) / v;
}
template <>
__device__ inline float fast_recip<float>(float v) {
  return __builtin_amdgcn_rcpf(v);  // 1 ulp; q only feeds a tolerance-checked sum
}

template <typename T>
__device__ inline T apply_prox(int prox, T z, T pw) {
  if (prox == 1) return z < T(0) ? T(0) : z;  // PositiveOrthant: clip(0, None)
  if (prox == 2) {                            // l1: fmax(0, |z| - pw) * sign(z)
    T m = fabs(z) - pw;
    m = m > T(0) ? m : T(0);
    T s = z > T(0) ? T(1) : (z < T(0) ? T(-1) : T(0));
    return m * s;
  }
  return z;
}

template <typename T, int R, bool TV, int PROX>
__global__ void __launch_bounds__(kThreads) pgd_tv2d_kernel(PgdParams<T> p, const T* __restrict__ x,
                                                            const T* __restrict__ xp, const T* __restrict__ y,
                                                            T* __restrict__ xn, double* __restrict__ partials) {
  using L = Layout<R>;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  T* A = reinterpret_cast<T*>(smem_raw);
  T* B = A + L::A_ELEMS;

  // XCD-aware tile order: blocks b and b+8 share an XCD; give each XCD a contiguous band.
  // Bijection: XCD group g = b % 8 owns q + (g < r) consecutive tiles starting at g*q + min(g, r).
  const int64_t nb = p.ntiles;
  const int64_t b = blockIdx.x;
  const int64_t q8 = nb / 8, r8 = nb % 8, g8 = b % 8;
  const int64_t tile = g8 * q8 + (g8 < r8 ? g8 : r8) + b / 8;
  const int64_t tpi = (int64_t)p.tiles0 * p.tiles1;
  const int64_t s = tile / tpi;
  const int64_t tr = tile - s * tpi;
  const int64_t ty0 = (tr / p.tiles1) * TY, tx0 = (tr % p.tiles1) * TX;
  const int64_t n0 = p.n0, n1 = p.n1;
  const T* xs = x + s * n0 * n1;
  const T* xps = xp + s * n0 * n1;
  const T* ys = y + (s % p.y_images) * n0 * n1;
  T* xns = xn + s * n0 * n1;

  // 1) yk on the (TY+4R) x (TX+4R) region, zero outside the image.
  for (int e = threadIdx.x; e < L::AR * L::AC; e += kThreads) {
    const int r = e / L::AC, c = e % L::AC;
    const int64_t gr = ty0 - 2 * R + r, gc = tx0 - 2 * R + c;
    T v = T(0);
    if (gr >= 0 && gr < n0 && gc >= 0 && gc < n1) {
      const int64_t g = gr * n1 + gc;
      const T xv = xs[g];
      T d = xv - xps[g];  // y = (x - x_prev) * a + x   (pgd.py:179-181)
      d = d * p.a;
      v = d + xv;
    }
    A[r * L::AP + c] = v;
  }
  __syncthreads();

  // Per-thread output strip (pass-D mapping): row rd, columns cd0 .. cd0 + SEG_D.
  const int rd = threadIdx.x / L::NSEG_D;
  const int cd0 = (threadIdx.x % L::NSEG_D) * L::SEG_D;
  T tv[L::SEG_D];
  T ykown[L::SEG_D];
#pragma unroll
  for (int i = 0; i < L::SEG_D; ++i) {
    ykown[i] = A[(rd + 2 * R) * L::AP + cd0 + i + 2 * R];
    tv[i] = T(0);
  }

  // 2) TV term: q on (TY+1) x (TX+1) into B, then Grad^T q at the thread's own pixels.
  if (TV) {
    T* Q0 = B;
    T* Q1 = B + L::QR * L::QP;
    for (int e = threadIdx.x; e < L::QR * L::QC; e += kThreads) {
      const int r = e / L::QC, c = e % L::QC;
      const int64_t gr = ty0 - 1 + r, gc = tx0 - 1 + c;
      T q0 = T(0), q1 = T(0);
      if (gr >= 0 && gr < n0 && gc >= 0 && gc < n1) {
        const int ar = r - 1 + 2 * R, ac = c - 1 + 2 * R;
        const T yc = A[ar * L::AP + ac];
        const T v0 = p.g0a * yc + p.g0b * A[(ar + 1) * L::AP + ac];
        const T v1 = p.g1a * yc + p.g1b * A[ar * L::AP + ac + 1];
        const T n = sqrt(v0 * v0 + v1 * v1);
        // (v - v (1 - mu / max(n, mu))) / mu * lam  ==  v * lam / max(n, mu)
        const T w = p.lam * fast_recip<T>(n > p.mu ? n : p.mu);
        q0 = v0 * w;
        q1 = v1 * w;
      }
      Q0[r * L::QP + c] = q0;
      Q1[r * L::QP + c] = q1;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < L::SEG_D; ++i) {
      const int r = rd + 1, c = cd0 + i + 1;
      // adjoint taps in flipped order: (+1 tap at i - e_d) then (-1 tap at i), summed over d
      T t0 = p.g0b * Q0[(r - 1) * L::QP + c] + p.g0a * Q0[r * L::QP + c];
      T t1 = p.g1b * Q1[r * L::QP + c - 1] + p.g1a * Q1[r * L::QP + c];
      tv[i] = t0 + t1;
    }
    __syncthreads();
  }

  // 3) H along axis 0: A (yk) -> B (P1)
  vpass<T, R, L::SEG_A>(A, L::AP, B, L::P1P, L::P1R, L::P1C, p.k0);
  __syncthreads();
  // 4) H along axis 1: B (P1) -> A (H yk), on the r region
  hpass<T, R, L::SEG_B>(B, L::P1P, A, L::AP, L::RR, L::RC, p.k1);
  __syncthreads();
  // 5) r = H yk - y inside the image, 0 outside (Trim^T zero-embedding of the residual)
  for (int e = threadIdx.x; e < L::RR * L::RC; e += kThreads) {
    const int r = e / L::RC, c = e % L::RC;
    const int64_t gr = ty0 - R + r, gc = tx0 - R + c;
    T v = T(0);
    if (gr >= 0 && gr < n0 && gc >= 0 && gc < n1) v = A[r * L::AP + c] - ys[gr * n1 + gc];
    A[r * L::AP + c] = v;
  }
  __syncthreads();
  // 6) H^T along axis 0 (flipped taps): A (r) -> B (P3)
  T kf0[2 * R + 1], kf1[2 * R + 1];
#pragma unroll
  for (int j = 0; j <= 2 * R; ++j) {
    kf0[j] = p.k0[2 * R - j];
    kf1[j] = p.k1[2 * R - j];
  }
  vpass<T, R, L::SEG_C>(A, L::AP, B, L::P3P, L::P3R, L::P3C, kf0);
  __syncthreads();

  // 7) H^T along axis 1 at the thread's own pixels, combine, prox, store.
  double part_d = 0.0, part_x = 0.0;
  {
    T win[L::SEG_D + 2 * R];
#pragma unroll
    for (int j = 0; j < L::SEG_D + 2 * R; ++j) win[j] = B[rd * L::P3P + cd0 + j];
    const int64_t gr = ty0 + rd;
#pragma unroll
    for (int i = 0; i < L::SEG_D; ++i) {
      T g = T(0);
#pragma unroll
      for (int j = 0; j <= 2 * R; ++j) g += kf1[j] * win[i + j];
      if (TV) g = g + tv[i];  // AddRule.grad: data term + TV term
      T z = g * (-p.tau);     // z = grad * (-tau) + y   (pgd.py:185-187)
      z = z + ykown[i];
      const T out = apply_prox<T>(PROX, z, p.pw);
      const int64_t gc = tx0 + cd0 + i;
      if (gr < n0 && gc < n1) {
        const int64_t g_idx = gr * n1 + gc;
        xns[g_idx] = out;
        if (partials) {
          const T xv = xs[g_idx];
          const double dd = (double)out - (double)xv;
          part_d += dd * dd;
          part_x += (double)xv * (double)xv;
        }
      }
    }
  }
  if (partials) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      part_d += __shfl_down(part_d, off, 64);
      part_x += __shfl_down(part_x, off, 64);
    }
    // reduction scratch after A and B in the dynamic LDS carve (no static __shared__ in front)
    double* red = reinterpret_cast<double*>(B + L::B_ELEMS + (L::B_ELEMS & 1));
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) {
      red[w] = part_d;
      red[kThreads / 64 + w] = part_x;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double a0 = 0, a1 = 0;
      for (int k = 0; k < kThreads / 64; ++k) {
        a0 += red[k];
        a1 += red[kThreads / 64 + k];
      }
      partials[2 * tile] = a0;
      partials[2 * tile + 1] = a1;
    }
  }
}

template <typename T, int R, bool TV, int PROX>
int launch_pgd(const PgdParams<T>& p, const void* x, const void* xp, const void* y, void* xn, double* partials,
               hipStream_t s) {
  using L = Layout<R>;
  size_t smem = (size_t)(L::A_ELEMS + L::B_ELEMS + 1) * sizeof(T) + 2 * (kThreads / 64) * sizeof(double) + 16;
  auto kern = pgd_tv2d_kernel<T, R, TV, PROX>;
  static bool configured = false;  // raise the dynamic-LDS cap once per instantiation
  if (!configured) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    configured = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)p.ntiles), dim3(kThreads), smem, s, p, (const T*)x, (const T*)xp,
                     (const T*)y, (T*)xn, partials);
  return last_launch_status();
}

template <typename T, int R>
int dispatch_flags(const PgdParams<T>& p, bool tv, int prox, const void* x, const void* xp, const void* y, void* xn,
                   double* partials, hipStream_t s) {
  if (tv) {
    if (prox == 0) return launch_pgd<T, R, true, 0>(p, x, xp, y, xn, partials, s);
    if (prox == 1) return launch_pgd<T, R, true, 1>(p, x, xp, y, xn, partials, s);
    return launch_pgd<T, R, true, 2>(p, x, xp, y, xn, partials, s);
  }
  if (prox == 0) return launch_pgd<T, R, false, 0>(p, x, xp, y, xn, partials, s);
  if (prox == 1) return launch_pgd<T, R, false, 1>(p, x, xp, y, xn, partials, s);
  return launch_pgd<T, R, false, 2>(p, x, xp, y, xn, partials, s);
}

template <typename T>
int pgd_entry(int64_t stack, int64_t y_images, int64_t n0, int64_t n1, int nt0, const int32_t* off0, const double* coef0, int nt1,
              const int32_t* off1, const double* coef1, double h0, double h1, double lam, double mu, double a,
              double tau, int prox, double prox_w, const void* x, const void* x_prev, const void* y, void* x_new,
              double* partials, hipStream_t s) {
  PXA_CHECK_ARG(stack >= 1 && n0 >= 1 && n1 >= 1 && y_images >= 1 && stack % y_images == 0);
  PXA_CHECK_ARG(x && x_prev && y && x_new);
  PXA_CHECK_ARG(x_new != x && x_new != x_prev);
  PXA_CHECK_ARG(prox >= 0 && prox <= 2);
  PXA_CHECK_ARG(nt0 >= 1 && nt1 >= 1 && off0 && off1 && coef0 && coef1);
  int R = 1;  // TV needs a 1-pixel halo even for a 1-tap blur
  for (int q = 0; q < nt0; ++q) R = abs(off0[q]) > R ? abs(off0[q]) : R;
  for (int q = 0; q < nt1; ++q) R = abs(off1[q]) > R ? abs(off1[q]) : R;
  if (R > kMaxR) return PXA_ERR_UNSUPPORTED;
  PgdParams<T> p;
  p.stack = stack;
  p.y_images = y_images;
  p.n0 = n0;
  p.n1 = n1;
  p.tiles0 = (int)((n0 + TY - 1) / TY);
  p.tiles1 = (int)((n1 + TX - 1) / TX);
  p.ntiles = stack * (int64_t)p.tiles0 * p.tiles1;
  PXA_CHECK_ARG(p.ntiles <= 0x7fffffff);
  for (int j = 0; j <= 2 * kMaxR; ++j) p.k0[j] = p.k1[j] = T(0);
  for (int q = 0; q < nt0; ++q) p.k0[off0[q] + R] += (T)coef0[q];
  for (int q = 0; q < nt1; ++q) p.k1[off1[q] + R] += (T)coef1[q];
  p.g0a = (T)(-1.0 / h0);
  p.g0b = (T)(1.0 / h0);
  p.g1a = (T)(-1.0 / h1);
  p.g1b = (T)(1.0 / h1);
  p.lam = (T)lam;
  p.mu = (T)mu;
  p.a = (T)a;
  p.tau = (T)tau;
  p.pw = (T)prox_w;
  bool tv = lam != 0.0;
  switch (R) {
    case 1: return dispatch_flags<T, 1>(p, tv, prox, x, x_prev, y, x_new, partials, s);
    case 2: return dispatch_flags<T, 2>(p, tv, prox, x, x_prev, y, x_new, partials, s);
    case 3: return dispatch_flags<T, 3>(p, tv, prox, x, x_prev, y, x_new, partials, s);
    case 4: return dispatch_flags<T, 4>(p, tv, prox, x, x_prev, y, x_new, partials, s);
    case 5: return dispatch_flags<T, 5>(p, tv, prox, x, x_prev, y, x_new, partials, s);
    case 6: return dispatch_flags<T, 6>(p, tv, prox, x, x_prev, y, x_new, partials, s);
    case 7: return dispatch_flags<T, 7>(p, tv, prox, x, x_prev, y, x_new, partials, s);
    default: return dispatch_flags<T, 8>(p, tv, prox, x, x_prev, y, x_new, partials, s);
  }
}

}  // namespace
}  // namespace pxa

using namespace pxa;

extern "C" {

int pxa_pgd_tv2d_partials_count(int64_t stack, int64_t n0, int64_t n1) {
  int64_t t = stack * ((n0 + TY - 1) / TY) * ((n1 + TX - 1) / TX);
  return (int)t;
}

int pxa_pgd_tv2d_step(int dtype, int64_t stack, int64_t y_images, int64_t n0, int64_t n1, int nt0, const int32_t* off0,
                      const double* coef0, int nt1, const int32_t* off1, const double* coef1, double h0, double h1,
                      double lam, double mu, double a, double tau, int prox, double prox_w, const void* x,
                      const void* x_prev, const void* y, void* x_new, double* partials, void* stream) {
  PXA_DISPATCH(dtype, T,
               return pgd_entry<T>(stack, y_images, n0, n1, nt0, off0, coef0, nt1, off1, coef1, h0, h1, lam, mu, a, tau, prox,
                                   prox_w, x, x_prev, y, x_new, partials, as_stream(stream)));
}

}  // extern "C"
