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
// One workgroup owns a TY x TX output tile and recomputes its halo in LDS.  HBM traffic per
// iteration is the compulsory 3 reads (x, x_prev, y) + 1 write (x_new) per pixel; halo re-reads
// hit L2 (tiles are dealt so that each XCD works on a contiguous band of the image).
//
// Work unit = a V x V block (V = elements per 16-B vector: 4 fp32, 2 fp64).  Every separable pass
// is a register-blocked sweep ALONG its stencil axis: a lane loads a (V+2R) x V window with
// ds_read_b128, forms V x V outputs with packed FMAs (v_pk_fma_f32 on the V-vector), and writes
// them TRANSPOSED, so the next pass (the other axis) again sweeps along rows of its input:
//
//   A   yk  row-major   rows [ty0-2R, ty0-2R+AR)   cols [tx0-CA, tx0-CA+AC)       (phase 0)
//   P1T H0 yk  [col][row]  cols = A cols          rows [ty0-R, ty0-R+P1R)        (pass 1, A -> P1T)
//   Rb  r = H1 P1 - y, row-major, rows = P1 rows  cols [tx0-R, tx0-R+RC)         (pass 2, P1T -> Rb, aliases A)
//   P3T H0^T r [col][row]  cols = Rb cols         rows [ty0, ty0+TY)             (pass 3, Rb -> P3T, aliases P1T)
//   out H1^T P3 + Grad^T q, prox                   rows [ty0, ty0+TY) cols [tx0, tx0+TX)  (pass 4)
//   Q   q0, q1 row-major  rows [ty0-1, ty0+TY)    cols [tx0-V, tx0+TX)            (from A, beside pass 1)
//
// Lane orders and LDS pitches are chosen with scripts/ldsbank.py (the MI355X_MICROARCH.md §LDS
// bank model: ds_read_b128 in four 16-lane groups on 64 banks, ds_write_b128 in 8-lane groups on
// 32 banks); for R = 6 every pass except pass 1 (+35 %) and the Q pass is at its conflict-free cost.
#include "common.hpp"

namespace pxa {
namespace {

constexpr int TY = 32;
constexpr int TX = 64;
constexpr int kThreads = 256;
constexpr int kMaxR = 8;

__host__ __device__ constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ constexpr int rup(int a, int b) { return cdiv(a, b) * b; }
__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }

template <typename T>
struct PgdParams {
  int64_t stack, n0, n1;
  int64_t y_images;  // y is shared by stack entries s with equal s % y_images
  int tiles0, tiles1;
  int64_t ntiles;  // stack * tiles0 * tiles1
  T k0[2 * kMaxR + 1], k1[2 * kMaxR + 1];  // H taps, dense window offsets -R..R (code-gen order)
  T g0a, g0b, g1a, g1b;                     // forward-difference taps per axis (-1/h, 1/h)
  T lam, mu, inv_mu, a, tau, pw;
  bool vec_ok;
};

template <typename T, int R>
struct Layout {
  static constexpr int V = kVecN<T>;  // elements per 16-B vector
  static constexpr bool F32 = sizeof(T) == 4;
  static constexpr int CA = rup(2 * R, V);        // A column halo, vector aligned
  static constexpr int P1R = rup(TY + 2 * R, V);  // rows of P1 / r
  static constexpr int AR = P1R + 2 * R, AC = TX + 2 * CA;
  static constexpr int RC = TX + CA;  // == rup(TX + 2R, V)
  static constexpr int QR = TY + 1, QC = TX + V;
  // V x V item grids
  static constexpr int NGA = AC / V;                       // phase 0: AR x NGA vectors
  static constexpr int NRG1 = P1R / V, NCG1 = AC / V;      // pass 1
  static constexpr int NSG2 = RC / V;                      // pass 2: NRG1 x NSG2
  static constexpr int NRG3 = TY / V, NCG3 = RC / V;       // pass 3
  static constexpr int NSG4 = TX / V;                      // pass 4: NRG3 x NSG4
  static constexpr int NQG = QC / V;                       // Q: QR x NQG vectors
  static constexpr int N0 = AR * NGA, N1 = NRG1 * NCG1, N3 = NRG3 * NCG3, N4 = NRG3 * NSG4, NQ = QR * NQG;
  static constexpr int N2P = rup(NRG1, 4) * rup(NSG2, 4);  // pass 2 uses padded 4 x 4 lane blocks
  // pitches (elements): fp32 residues from the bank model, fp64 dense
  static constexpr int pad(int w, int m, int res) {
    int p = w;
    while ((p % m) != res) p += V;
    return p;
  }
  static constexpr int AP = AC;  // ≡ 12 (mod 16) would make pass 1 conflict-free but costs a WG/CU
  static constexpr int PT = F32 ? pad(P1R, 8, 4) : P1R;
  static constexpr int RP = F32 ? pad(RC, 16, 12) : RC;
  static constexpr int P3P = F32 ? pad(TY, 8, 4) : TY;
  static constexpr int QP = F32 ? pad(QC, 16, 4) : QC;
  static constexpr int E_A = cmax(AR * AP, P1R * RP);
  static constexpr int E_T = cmax(AC * PT, RC * P3P);
  static constexpr int E_Q = 2 * QR * QP;
  // (the partial-sum scratch reuses Tb after the last pass).  NB: gfx950 allocates LDS in 2 KiB
  // granules per workgroup: 3 workgroups/CU need <= 52 KiB, 4 need <= 40 KiB.
  static constexpr size_t BYTES = (size_t)(E_A + E_T + E_Q) * sizeof(T);
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

// q = lam * v / max(|v|, mu)  ==  lam (v - prox_{mu L21}(v)) / mu; returns the scalar weight.
template <typename T>
__device__ inline T tv_weight(T n2, T lam, T mu, T inv_mu) {
  return lam / (sqrt(n2) > mu ? sqrt(n2) : mu);
}
template <>
__device__ inline float tv_weight<float>(float n2, float lam, float mu, float inv_mu) {
  const float r = __builtin_amdgcn_rsqf(n2);  // 1/|v| (inf at 0), 1 ulp
  return lam * (r < inv_mu ? r : inv_mu);
}

template <typename T>
__device__ inline T apply_prox(int prox, T z, T pw) {
  if (prox == 1) return fmax(z, T(0));  // PositiveOrthant: clip(0, None) (v_max; finite inputs)
  if (prox == 2) {                            // L1: sign(z) * max(|z| - pw, 0)
    T m = (z < T(0) ? -z : z) - pw;
    m = m > T(0) ? m : T(0);
    return z < T(0) ? -m : m;
  }
  return z;
}

// Lane orders (item id -> (a, b) with a the row-group-like and b the column-group-like index).
// a4: runs of 4 consecutive a per b, blocks of 4 a-rows; a: a fastest; blk: padded 4 x 4 blocks.
template <int NA, int NB>
__device__ inline void ord_a4(int it, int& a, int& b) {
  const int a0 = (it / (4 * NB)) * 4;
  const int rem = it - a0 * NB;
  if (NA % 4 == 0 || a0 + 4 <= NA) {
    b = rem >> 2;
    a = a0 + (rem & 3);
  } else {
    constexpr int hl = NA % 4 == 0 ? 4 : NA % 4;
    b = rem / hl;
    a = a0 + rem % hl;
  }
}
template <int NA, int NB>
__device__ inline void ord_a(int it, int& a, int& b) {
  b = it / NA;
  a = it - b * NA;
}
template <int NA, int NB>
__device__ inline bool ord_blk(int it, int& a, int& b) {
  constexpr int NBB = cdiv(NB, 4);
  const int blk = it >> 4, l = it & 15;
  const int ab = blk / NBB;
  a = ab * 4 + (l & 3);
  b = (blk - ab * NBB) * 4 + (l >> 2);
  return a < NA && b < NB;
}

// Packed-arithmetic unit: fp32 pairs (v_pk_fma_f32), fp64 scalars.
template <typename T>
struct Pk {
  using type = T;
  static constexpr int W = 1;
  __device__ static type splat(T v) { return v; }
};
template <>
struct Pk<float> {
  typedef float type __attribute__((ext_vector_type(2)));
  static constexpr int W = 2;
  __device__ static type splat(float v) { return type{v, v}; }
};

// Sweep along the leading (stencil) axis of a [m][V]-strided source: out[i][v] = sum_j k[j] *
// src[(i + j) * PS + v], i < V, from a (V + 2R) x V window.  FLIP reads the taps reversed (H^T).
// The FMAs are written on explicit pairs along v so that they pack as loaded (no operand moves).
template <typename T, int R, int PS, bool FLIP>
__device__ inline void sweep(const T* __restrict__ src, const T* __restrict__ k, T (&acc)[kVecN<T>][kVecN<T>]) {
  constexpr int V = kVecN<T>;
  using P = typename Pk<T>::type;
  constexpr int W = Pk<T>::W, NP = V / W;
  using VT = typename Vec4<T>::type;
  P win[V + 2 * R][NP];
#pragma unroll
  for (int j = 0; j < V + 2 * R; ++j) {
    const VT t = *reinterpret_cast<const VT*>(src + j * PS);
    __builtin_memcpy(&win[j][0], &t, sizeof(VT));
  }
  P a[V][NP];
#pragma unroll
  for (int i = 0; i < V; ++i)
#pragma unroll
    for (int h = 0; h < NP; ++h) a[i][h] = Pk<T>::splat(T(0));
#pragma unroll
  for (int j = 0; j <= 2 * R; ++j) {
    const P kk = Pk<T>::splat(FLIP ? k[2 * R - j] : k[j]);
#pragma unroll
    for (int i = 0; i < V; ++i)
#pragma unroll
      for (int h = 0; h < NP; ++h) a[i][h] = kk * win[i + j][h] + a[i][h];
  }
#pragma unroll
  for (int i = 0; i < V; ++i) __builtin_memcpy(&acc[i][0], &a[i][0], sizeof(T) * V);
}

// Transposed V x V store: dst[v * PD + i] = acc[i][v].
template <typename T, int PD>
__device__ inline void store_t(T* __restrict__ dst, const T (&acc)[kVecN<T>][kVecN<T>]) {
  constexpr int V = kVecN<T>;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    T col[V];
#pragma unroll
    for (int i = 0; i < V; ++i) col[i] = acc[i][v];
    st_vec<T, V>(dst + v * PD, col);
  }
}

// Global V-vector load at an element offset whose alignment is known at compile time (MIS = the
// offset mod V): one 16-B load, two 8-B loads (fp32, even offset) or scalars.
template <typename T, int MIS>
__device__ inline void ld_row(const T* __restrict__ p, T (&v)[kVecN<T>]) {
  constexpr int V = kVecN<T>;
  if constexpr (MIS == 0) {
    ld_vec<T, V>(p, v);
  } else if constexpr (sizeof(T) == 4 && (MIS % 2) == 0) {
    const float2 lo = *reinterpret_cast<const float2*>(p);
    const float2 hi = *reinterpret_cast<const float2*>(p + 2);
    v[0] = lo.x;
    v[1] = lo.y;
    v[2] = hi.x;
    v[3] = hi.y;
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = p[i];
  }
}

template <typename T, int R, bool TV, int PROX, bool EDGE>
__device__ inline void pgd_tile(const PgdParams<T>& p, unsigned char* smem, int64_t tile, int ty0, int tx0,
                                const T* __restrict__ xs, const T* __restrict__ xps, const T* __restrict__ ys,
                                T* __restrict__ xns, double* __restrict__ partials) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
  constexpr int CA = L::CA;
  T* A = reinterpret_cast<T*>(smem);   // yk, later Rb
  T* Tb = A + L::E_A;                  // P1T, later P3T
  T* Q0 = Tb + L::E_T;
  T* Q1 = Q0 + L::QR * L::QP;
  double* red = reinterpret_cast<double*>(Tb);
  T* Rb = A;
  const int n0 = (int)p.n0, n1 = (int)p.n1;
  const int tid = threadIdx.x;

  // ---- phase 0: yk = (x - x_prev) * a + x on A, zero outside the image  (pgd.py:179-181)
  constexpr int K0 = cdiv(L::N0, kThreads);
#pragma unroll
  for (int k = 0; k < K0; ++k) {
    const int it = tid + k * kThreads;
    if (it < L::N0) {
      const int r = it / L::NGA, g = it - r * L::NGA;
      const int gr = ty0 - 2 * R + r, gc = tx0 - CA + V * g;
      T xv[V], pv[V], out[V];
      if (!EDGE) {
        const unsigned off = (unsigned)(gr * n1 + gc);
        ld_vec<T, V>(xs + off, xv);
        ld_vec<T, V>(xps + off, pv);
      } else if (gr >= 0 && gr < n0 && p.vec_ok && gc >= 0 && gc + V <= n1) {
        ld_vec<T, V>(xs + (int64_t)gr * n1 + gc, xv);
        ld_vec<T, V>(xps + (int64_t)gr * n1 + gc, pv);
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const bool in = gr >= 0 && gr < n0 && gc + v >= 0 && gc + v < n1;
          xv[v] = in ? xs[(int64_t)gr * n1 + gc + v] : T(0);
          pv[v] = in ? xps[(int64_t)gr * n1 + gc + v] : T(0);
        }
      }
#pragma unroll
      for (int v = 0; v < V; ++v) {
        T d = xv[v] - pv[v];
        d = d * p.a;
        out[v] = d + xv[v];
      }
      st_vec<T, V>(A + r * L::AP + V * g, out);
    }
  }

  // prefetch y for pass 2 (global latency overlaps the Q / pass-1 phase)
  constexpr int K2 = cdiv(L::N2P, kThreads);
  T yv[K2][V][V];
#pragma unroll
  for (int k = 0; k < K2; ++k) {
    int a, b;
    const bool ok = ord_blk<L::NRG1, L::NSG2>(tid + k * kThreads, a, b) && (tid + k * kThreads < L::N2P);
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const int gr = ty0 - R + V * a + u, gc = tx0 - R + V * b;
      if (!EDGE) {
        if (ok) ld_row<T, ((V - R % V) % V)>(ys + (unsigned)(gr * n1 + gc), yv[k][u]);
      } else {
#pragma unroll
        for (int c = 0; c < V; ++c) {
          const bool in = ok && gr >= 0 && gr < n0 && gc + c >= 0 && gc + c < n1;
          yv[k][u][c] = in ? ys[(int64_t)gr * n1 + gc + c] : T(0);
        }
      }
    }
  }
  __syncthreads();

  // ---- Q: Moreau-TV dual field from yk; owned yk for the final combine; pass 1 (H along axis 0)
  if (TV) {
    constexpr int KQ = cdiv(L::NQ, kThreads);
#pragma unroll
    for (int k = 0; k < KQ; ++k) {
      const int it = tid + k * kThreads;
      if (it < L::NQ) {
        int r, g;
        ord_a<L::QR, L::NQG>(it, r, g);
        const int arow = r - 1 + 2 * R, acol = V * g + CA - V;
        T y0[V], y1[V], q0[V], q1[V];
        ld_vec<T, V>(A + arow * L::AP + acol, y0);
        ld_vec<T, V>(A + (arow + 1) * L::AP + acol, y1);
        const T yr = A[arow * L::AP + acol + V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const T yn = v + 1 < V ? y0[v + 1] : yr;
          const T v0 = p.g0a * y0[v] + p.g0b * y1[v];
          const T v1 = p.g1a * y0[v] + p.g1b * yn;
          T w = tv_weight<T>(v0 * v0 + v1 * v1, p.lam, p.mu, p.inv_mu);
          if (EDGE) {
            const int gr = ty0 - 1 + r, gc = tx0 - V + V * g + v;
            if (!(gr >= 0 && gr < n0 && gc >= 0 && gc < n1)) w = T(0);
          }
          q0[v] = v0 * w;
          q1[v] = v1 * w;
        }
        st_vec<T, V>(Q0 + r * L::QP + V * g, q0);
        st_vec<T, V>(Q1 + r * L::QP + V * g, q1);
      }
    }
  }
  constexpr int K4 = cdiv(L::N4, kThreads);
  T ykown[K4][V][V];
#pragma unroll
  for (int k = 0; k < K4; ++k) {
    const int it = tid + k * kThreads;
    if (it < L::N4) {
      int a, b;
      ord_a<L::NRG3, L::NSG4>(it, a, b);
#pragma unroll
      for (int u = 0; u < V; ++u) ld_vec<T, V>(A + (V * a + u + 2 * R) * L::AP + CA + V * b, ykown[k][u]);
    }
  }
  constexpr int K1 = cdiv(L::N1, kThreads);
#pragma unroll
  for (int k = 0; k < K1; ++k) {
    const int it = tid + k * kThreads;
    if (it < L::N1) {
      int a, b;
      ord_a4<L::NRG1, L::NCG1>(it, a, b);
      T acc[V][V];
      sweep<T, R, L::AP, false>(A + (V * a) * L::AP + V * b, p.k0, acc);
      store_t<T, L::PT>(Tb + (V * b) * L::PT + V * a, acc);
    }
  }
  __syncthreads();

  // ---- pass 2: H along axis 1, minus y, zero outside the image: P1T -> Rb (row-major)
#pragma unroll
  for (int k = 0; k < K2; ++k) {
    const int it = tid + k * kThreads;
    int a, b;
    if (it < L::N2P && ord_blk<L::NRG1, L::NSG2>(it, a, b)) {
      T acc[V][V];  // acc[c][u]: column c of the segment, row u of the group
      sweep<T, R, L::PT, false>(Tb + (V * b + CA - 2 * R) * L::PT + V * a, p.k1, acc);
#pragma unroll
      for (int u = 0; u < V; ++u) {
        T row[V];
#pragma unroll
        for (int c = 0; c < V; ++c) {
          T rv = acc[c][u] - yv[k][u][c];
          if (EDGE) {
            const int gr = ty0 - R + V * a + u, gc = tx0 - R + V * b + c;
            if (!(gr >= 0 && gr < n0 && gc >= 0 && gc < n1)) rv = T(0);
          }
          row[c] = rv;
        }
        st_vec<T, V>(Rb + (V * a + u) * L::RP + V * b, row);
      }
    }
  }
  __syncthreads();

  // ---- pass 3: H^T along axis 0 (flipped taps): Rb -> P3T
  constexpr int K3 = cdiv(L::N3, kThreads);
#pragma unroll
  for (int k = 0; k < K3; ++k) {
    const int it = tid + k * kThreads;
    if (it < L::N3) {
      int a, b;
      ord_a<L::NRG3, L::NCG3>(it, a, b);
      T acc[V][V];
      sweep<T, R, L::RP, true>(Rb + (V * a) * L::RP + V * b, p.k0, acc);
      store_t<T, L::P3P>(Tb + (V * b) * L::P3P + V * a, acc);
    }
  }
  __syncthreads();

  // ---- pass 4: H^T along axis 1 + Grad^T q; z = grad * (-tau) + yk; prox; store  (pgd.py:185-191)
  double part_d = 0.0, part_x = 0.0;
#pragma unroll
  for (int k = 0; k < K4; ++k) {
    const int it = tid + k * kThreads;
    if (it < L::N4) {
      int a, b;
      ord_a<L::NRG3, L::NSG4>(it, a, b);
      T acc[V][V];  // acc[c][u]
      sweep<T, R, L::P3P, true>(Tb + (V * b) * L::P3P + V * a, p.k1, acc);
      T tv[V][V];  // tv[u][c]
      if (TV) {
        T q0r[V + 1][V];
#pragma unroll
        for (int u = 0; u <= V; ++u) ld_vec<T, V>(Q0 + (V * a + u) * L::QP + V * b + V, q0r[u]);
#pragma unroll
        for (int u = 0; u < V; ++u) {
          T lo[V], hi[V];
          ld_vec<T, V>(Q1 + (V * a + u + 1) * L::QP + V * b, lo);
          ld_vec<T, V>(Q1 + (V * a + u + 1) * L::QP + V * b + V, hi);
#pragma unroll
          for (int c = 0; c < V; ++c) {
            const T q1m = c == 0 ? lo[V - 1] : hi[c - 1];
            // Grad^T q: flipped 2-tap adjoints, (+1 tap at i - e_d) then (-1 tap at i), summed over d
            const T t0 = p.g0b * q0r[u][c] + p.g0a * q0r[u + 1][c];
            const T t1 = p.g1b * q1m + p.g1a * hi[c];
            tv[u][c] = t0 + t1;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < V; ++u) {
        T out[V];
#pragma unroll
        for (int c = 0; c < V; ++c) {
          const T gsum = TV ? acc[c][u] + tv[u][c] : acc[c][u];  // AddRule.grad: data + TV
          T z = gsum * (-p.tau);
          z = z + ykown[k][u][c];
          out[c] = apply_prox<T>(PROX, z, p.pw);
        }
        const int gr = ty0 + V * a + u, gc = tx0 + V * b;
        if (!EDGE) {
          const unsigned off = (unsigned)(gr * n1 + gc);
          st_vec<T, V>(xns + off, out);
          if (partials) {
            T xv[V];
            ld_vec<T, V>(xs + off, xv);
#pragma unroll
            for (int c = 0; c < V; ++c) {
              const double dd = (double)out[c] - (double)xv[c];
              part_d += dd * dd;
              part_x += (double)xv[c] * (double)xv[c];
            }
          }
        } else if (gr < n0) {
#pragma unroll
          for (int c = 0; c < V; ++c) {
            if (gc + c < n1) {
              xns[(int64_t)gr * n1 + gc + c] = out[c];
              if (partials) {
                const T xv = xs[(int64_t)gr * n1 + gc + c];
                const double dd = (double)out[c] - (double)xv;
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
    const int lane = tid & 63, w = tid >> 6;
    __syncthreads();  // Tb (P3T) is free again
    if (lane == 0) {
      red[w] = part_d;
      red[kThreads / 64 + w] = part_x;
    }
    __syncthreads();
    if (tid == 0) {
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
__global__ void __launch_bounds__(kThreads) pgd_tv2d_kernel(PgdParams<T> p, const T* __restrict__ x,
                                                            const T* __restrict__ xp, const T* __restrict__ y,
                                                            T* __restrict__ xn, double* __restrict__ partials) {
  using L = Layout<T, R>;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  // XCD-aware tile order (speed only): XCD group g = b % 8 owns a contiguous band of tiles.
  // (ntiles < 2^31 is checked on the host: 32-bit index math.)
  const unsigned nb = (unsigned)p.ntiles;
  const unsigned b = blockIdx.x;
  const unsigned q8 = nb >> 3, r8 = nb & 7u, g8 = b & 7u;
  const unsigned tile = g8 * q8 + (g8 < r8 ? g8 : r8) + (b >> 3);
  const unsigned tpi = (unsigned)p.tiles0 * (unsigned)p.tiles1;
  const unsigned s = tile / tpi;
  const unsigned tr = tile - s * tpi;
  const unsigned trow = tr / (unsigned)p.tiles1;
  const int ty0 = (int)trow * TY, tx0 = (int)(tr - trow * (unsigned)p.tiles1) * TX;
  const int64_t img = p.n0 * p.n1;
  const T* xs = x + (int64_t)s * img;
  const T* xps = xp + (int64_t)s * img;
  const T* ys = y + (int64_t)(s % (unsigned)p.y_images) * img;
  T* xns = xn + (int64_t)s * img;
  // interior: the whole A window lies inside the image and rows are 16-B aligned -> no bounds tests
  const bool interior = p.vec_ok && img <= 0x7fffffff && ty0 - 2 * R >= 0 && ty0 - 2 * R + L::AR <= p.n0 && tx0 - L::CA >= 0 &&
                        tx0 - L::CA + L::AC <= p.n1;
  if (interior)
    pgd_tile<T, R, TV, PROX, false>(p, smem_raw, tile, ty0, tx0, xs, xps, ys, xns, partials);
  else
    pgd_tile<T, R, TV, PROX, true>(p, smem_raw, tile, ty0, tx0, xs, xps, ys, xns, partials);
}

template <typename T, int R, bool TV, int PROX>
int launch_pgd(const PgdParams<T>& p, const void* x, const void* xp, const void* y, void* xn, double* partials,
               hipStream_t s) {
  using L = Layout<T, R>;
  const size_t smem = L::BYTES;
  auto kern = pgd_tv2d_kernel<T, R, TV, PROX>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr_set = true;
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
  p.inv_mu = (T)(1.0 / mu);
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
