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
  bool vec_ok;
};

// Geometry (R: blur radius along rows; RA: R rounded up to the 16-B vector width along columns so
// every horizontal window starts on an aligned LDS address):
//   A  (yk)  rows [ty0-2R, ty0+TY+2R)  cols [tx0-2RA, tx0+TX+2RA)
//   P1       rows [ty0-R,  ty0+TY+R)   cols  = A cols                 (H along axis 0)
//   r        rows  = P1 rows           cols [tx0-RA, tx0+TX+RA)       (H along axis 1, - y; in A)
//   P3       rows [ty0, ty0+TY)        cols  = r cols                 (H^T along axis 0; in B)
//   out      rows [ty0, ty0+TY)        cols [tx0, tx0+TX)             (H^T along axis 1)
//   Q (q0,q1) rows [ty0-1, ty0+TY)     cols [tx0-1, tx0+TX)           (Moreau-TV dual field; in B)
template <typename T, int R>
struct Layout {
  static constexpr int V = kVecN<T>;                  // elements per 16-B vector
  static constexpr int RA = (R + V - 1) / V * V;
  static constexpr int AR = TY + 4 * R, AC = TX + 4 * RA;
  static constexpr int P1R = TY + 2 * R, P1C = AC;
  static constexpr int RR = TY + 2 * R, RC = TX + 2 * RA;
  static constexpr int P3R = TY, P3C = RC;
  static constexpr int QR = TY + 1, QC = TX + 1, QP = TX + 1 + (((TX + 1) & 1) ? 0 : 1);
  static constexpr int A_ELEMS = AR * AC;
  static constexpr int B_ELEMS_Q = 2 * QR * QP;
  static constexpr int B_ELEMS = (P1R * P1C > B_ELEMS_Q) ? P1R * P1C : B_ELEMS_Q;
  // vector groups per row and strip lengths sized to ~one item per thread
  static constexpr int GA = AC / V, GR = RC / V, GO = TX / V;
  static constexpr int NSEG_A = kThreads / GA > 0 ? kThreads / GA : 1;
  static constexpr int SEG_A = cdiv(P1R, NSEG_A);
  static constexpr int NSEG_C = kThreads / GR > 0 ? kThreads / GR : 1;
  static constexpr int SEG_C = cdiv(P3R, NSEG_C);
  static constexpr int ITEMS_D = TY * GO;                 // pass-D items (V outputs each)
  static constexpr int PER_D = cdiv(ITEMS_D, kThreads);  // items per thread in pass D
};

template <typename T>
struct VecT {
  using type = typename Vec4<T>::type;
};

template <typename T, int V>
__device__ inline void ld_vec(const T* p, T (&v)[V]) {
  using VT = typename Vec4<T>::type;
  *reinterpret_cast<VT*>(v) = *reinterpret_cast<const VT*>(p);
}
template <typename T, int V>
__device__ inline void st_vec(T* p, const T (&v)[V]) {
  using VT = typename Vec4<T>::type;
  *reinterpret_cast<VT*>(p) = *reinterpret_cast<const VT*>(v);
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

// Vertical (axis-0) pass over vector groups: dst[r][c] = sum_j k[j] src[r + j][c], r < NR, all GROUPS.
template <typename T, int R, int SEG, int NR, int GROUPS, int PS, int PD>
__device__ inline void vpass(const T* __restrict__ src, T* __restrict__ dst, const T* __restrict__ k) {
  constexpr int V = kVecN<T>;
  constexpr int NSEG = cdiv(NR, SEG);
  constexpr int ITEMS = GROUPS * NSEG;
  for (int item = threadIdx.x; item < ITEMS; item += kThreads) {
    const int g = item % GROUPS, r0 = (item / GROUPS) * SEG;
    T win[SEG + 2 * R][V];
#pragma unroll
    for (int j = 0; j < SEG + 2 * R; ++j) {
      if (r0 + j < NR + 2 * R) {
        ld_vec<T, V>(src + (r0 + j) * PS + g * V, win[j]);
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) win[j][v] = T(0);
      }
    }
#pragma unroll
    for (int i = 0; i < SEG; ++i) {
      if (r0 + i < NR) {
        T acc[V];
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] = T(0);
#pragma unroll
        for (int j = 0; j <= 2 * R; ++j)
#pragma unroll
          for (int v = 0; v < V; ++v) acc[v] += k[j] * win[i + j][v];
        st_vec<T, V>(dst + (r0 + i) * PD + g * V, acc);
      }
    }
  }
}

// Horizontal (axis-1) correlation of one vector group: out[v] = sum_o k[o+R] src[RA + o + v], the
// window src[0 .. V + 2RA) starting on an aligned address.
template <typename T, int R>
__device__ inline void hgroup(const T* __restrict__ src, const T* __restrict__ k, T (&out)[kVecN<T>]) {
  constexpr int V = kVecN<T>;
  constexpr int RA = (R + V - 1) / V * V;
  constexpr int W = V + 2 * RA;
  T win[W];
#pragma unroll
  for (int j = 0; j < W / V; ++j) {
    T tmp[V];
    ld_vec<T, V>(src + j * V, tmp);
#pragma unroll
    for (int v = 0; v < V; ++v) win[j * V + v] = tmp[v];
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {
    T acc = T(0);
#pragma unroll
    for (int j = 0; j <= 2 * R; ++j) acc += k[j] * win[RA - R + j + v];
    out[v] = acc;
  }
}

template <typename T, int R, bool TV, int PROX>
__global__ void __launch_bounds__(kThreads) pgd_tv2d_kernel(PgdParams<T> p, const T* __restrict__ x,
                                                            const T* __restrict__ xp, const T* __restrict__ y,
                                                            T* __restrict__ xn, double* __restrict__ partials) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
  constexpr int RA = L::RA;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  T* A = reinterpret_cast<T*>(smem_raw);
  T* B = A + L::A_ELEMS;

  // XCD-aware tile order (speed only): XCD group g = b % 8 owns a contiguous band of tiles.
  const int64_t nb = p.ntiles;
  const int64_t b = blockIdx.x;
  const int64_t q8 = nb / 8, r8 = nb % 8, g8 = b % 8;
  const int64_t tile = g8 * q8 + (g8 < r8 ? g8 : r8) + b / 8;
  const int64_t tpi = (int64_t)p.tiles0 * p.tiles1;
  const int64_t s = tile / tpi;
  const int tr = (int)(tile - s * tpi);
  const int ty0 = (tr / p.tiles1) * TY, tx0 = (tr % p.tiles1) * TX;
  const int n0 = (int)p.n0, n1 = (int)p.n1;
  const int64_t img = (int64_t)n0 * n1;
  const T* __restrict__ xs = x + s * img;
  const T* __restrict__ xps = xp + s * img;
  const T* __restrict__ ys = y + (s % p.y_images) * img;
  T* __restrict__ xns = xn + s * img;
  const bool vec_ok = p.vec_ok;  // rows are 16-B aligned (n1 % V == 0, aligned bases)

  // 1) yk = (x - x_prev) * a + x on A, zero outside the image.
  for (int e = threadIdx.x; e < L::AR * L::GA; e += kThreads) {
    const int r = e / L::GA, g = e % L::GA;
    const int gr = ty0 - 2 * R + r, gc = tx0 - 2 * RA + g * V;
    T xv[V], pv[V], out[V];
    if (gr >= 0 && gr < n0 && vec_ok && gc >= 0 && gc + V <= n1) {
      ld_vec<T, V>(xs + gr * n1 + gc, xv);
      ld_vec<T, V>(xps + gr * n1 + gc, pv);
    } else {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const bool in = gr >= 0 && gr < n0 && gc + v >= 0 && gc + v < n1;
        xv[v] = in ? xs[gr * n1 + gc + v] : T(0);
        pv[v] = in ? xps[gr * n1 + gc + v] : T(0);
      }
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
      T d = xv[v] - pv[v];  // (x - x_prev) * a + x   (pgd.py:179-181)
      d = d * p.a;
      out[v] = d + xv[v];
    }
    st_vec<T, V>(A + r * L::AC + g * V, out);
  }
  __syncthreads();

  // Thread-owned output groups (pass-D mapping): item it -> row it / GO, group it % GO.
  T ykown[L::PER_D][V];
  T tv[L::PER_D][V];
#pragma unroll
  for (int k = 0; k < L::PER_D; ++k) {
    const int it = threadIdx.x + k * kThreads;
#pragma unroll
    for (int v = 0; v < V; ++v) tv[k][v] = T(0);
    if (it < L::ITEMS_D) {
      const int r = it / L::GO, g = it % L::GO;
      ld_vec<T, V>(A + (r + 2 * R) * L::AC + 2 * RA + g * V, ykown[k]);
    }
  }

  // 2) Moreau-TV: q on (TY+1) x (TX+1) into B, then Grad^T q at the owned pixels.
  if (TV) {
    T* Q0 = B;
    T* Q1 = B + L::QR * L::QP;
    for (int e = threadIdx.x; e < L::QR * L::QC; e += kThreads) {
      const int r = e / L::QC, c = e % L::QC;
      const int gr = ty0 - 1 + r, gc = tx0 - 1 + c;
      T q0 = T(0), q1 = T(0);
      if (gr >= 0 && gr < n0 && gc >= 0 && gc < n1) {
        const int ar = r - 1 + 2 * R, ac = c - 1 + 2 * RA;
        const T yc = A[ar * L::AC + ac];
        const T v0 = p.g0a * yc + p.g0b * A[(ar + 1) * L::AC + ac];
        const T v1 = p.g1a * yc + p.g1b * A[ar * L::AC + ac + 1];
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
    for (int k = 0; k < L::PER_D; ++k) {
      const int it = threadIdx.x + k * kThreads;
      if (it < L::ITEMS_D) {
        const int r = it / L::GO + 1, c0 = (it % L::GO) * V + 1;
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const int c = c0 + v;
          // flipped adjoint taps: (+1 tap at i - e_d) then (-1 tap at i), summed over d
          const T t0 = p.g0b * Q0[(r - 1) * L::QP + c] + p.g0a * Q0[r * L::QP + c];
          const T t1 = p.g1b * Q1[r * L::QP + c - 1] + p.g1a * Q1[r * L::QP + c];
          tv[k][v] = t0 + t1;
        }
      }
    }
    __syncthreads();
  }

  // 3) H along axis 0: A (yk) -> B (P1)
  vpass<T, R, L::SEG_A, L::P1R, L::GA, L::AC, L::P1C>(A, B, p.k0);
  __syncthreads();

  // 4) H along axis 1 on the r region, r = H yk - y inside the image, 0 outside: B (P1) -> A (r)
  for (int e = threadIdx.x; e < L::RR * L::GR; e += kThreads) {
    const int r = e / L::GR, g = e % L::GR;
    T hv[V], yv[V];
    hgroup<T, R>(B + r * L::P1C + g * V, p.k1, hv);
    const int gr = ty0 - R + r, gc = tx0 - RA + g * V;
    if (gr >= 0 && gr < n0 && vec_ok && gc >= 0 && gc + V <= n1) {
      ld_vec<T, V>(ys + gr * n1 + gc, yv);
#pragma unroll
      for (int v = 0; v < V; ++v) hv[v] = hv[v] - yv[v];
    } else {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const bool in = gr >= 0 && gr < n0 && gc + v >= 0 && gc + v < n1;
        hv[v] = in ? hv[v] - ys[gr * n1 + gc + v] : T(0);
      }
    }
    st_vec<T, V>(A + r * L::RC + g * V, hv);
  }
  __syncthreads();

  // 5) H^T along axis 0 (flipped taps): A (r) -> B (P3)
  T kf0[2 * R + 1], kf1[2 * R + 1];
#pragma unroll
  for (int j = 0; j <= 2 * R; ++j) {
    kf0[j] = p.k0[2 * R - j];
    kf1[j] = p.k1[2 * R - j];
  }
  vpass<T, R, L::SEG_C, L::P3R, L::GR, L::RC, L::P3C>(A, B, kf0);
  __syncthreads();

  // 6) H^T along axis 1 at the owned pixels; grad = data + TV; z = grad * (-tau) + yk; prox; store.
  double part_d = 0.0, part_x = 0.0;
#pragma unroll
  for (int k = 0; k < L::PER_D; ++k) {
    const int it = threadIdx.x + k * kThreads;
    if (it < L::ITEMS_D) {
      const int r = it / L::GO, g = it % L::GO;
      T gv[V], out[V];
      hgroup<T, R>(B + r * L::P3C + g * V, kf1, gv);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        T gr_ = TV ? gv[v] + tv[k][v] : gv[v];  // AddRule.grad: data term + TV term
        T z = gr_ * (-p.tau);                   // z = grad * (-tau) + y   (pgd.py:185-187)
        z = z + ykown[k][v];
        out[v] = apply_prox<T>(PROX, z, p.pw);
      }
      const int gr = ty0 + r, gc = tx0 + g * V;
      if (gr < n0) {
        if (vec_ok && gc + V <= n1) {
          st_vec<T, V>(xns + gr * n1 + gc, out);
          if (partials) {
            T xv[V];
            ld_vec<T, V>(xs + gr * n1 + gc, xv);
#pragma unroll
            for (int v = 0; v < V; ++v) {
              const double dd = (double)out[v] - (double)xv[v];
              part_d += dd * dd;
              part_x += (double)xv[v] * (double)xv[v];
            }
          }
        } else {
#pragma unroll
          for (int v = 0; v < V; ++v) {
            if (gc + v < n1) {
              xns[gr * n1 + gc + v] = out[v];
              if (partials) {
                const T xv = xs[gr * n1 + gc + v];
                const double dd = (double)out[v] - (double)xv;
                part_d += dd * dd;
                part_x += (double)xv * (double)xv;
              }
            }
          }
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
    __syncthreads();  // B is free again: reuse it for the cross-wave sums
    double* red = reinterpret_cast<double*>(B);
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
  using L = Layout<T, R>;
  size_t smem = (size_t)(L::A_ELEMS + L::B_ELEMS) * sizeof(T);
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
  constexpr int V = kVecN<T>;
  p.vec_ok = (n1 % V == 0) && aligned16(x) && aligned16(x_prev) && aligned16(y) && aligned16(x_new);
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
