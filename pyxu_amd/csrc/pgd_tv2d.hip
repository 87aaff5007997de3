// Fused PGD step for 2-D TV-regularised deblurring, normal-operator form: one launch per iteration.
//
//   yk     = x + a (x - x_prev)                                            (pgd.py:179-181)
//   grad   = (G yk - b) + Grad^T q,   G = H^T H,  b = H^T y  (b precomputed once per solve)
//   q      = lam * v / max(|v|, mu)  ==  lam (v - prox_{mu L21}(v)) / mu,  v = Grad yk
//   x_new  = prox_{tau g}( grad * (-tau) + yk )                            (pgd.py:185-191)
//
// Reference dataflow: PGD.m_step (opt/solver/pgd.py:173-191) through AddRule.grad,
// ChainRule.grad, ScaleRule.grad, ArgShiftRule.grad (abc/arithmetic.py), Stencil.apply/adjoint
// (operator/linop/stencil/stencil.py:441-461), Gradient (operator/linop/diff.py:1113-1265), the
// moreau_envelope gradient (abc/operator.py:1053-1058), L21Norm.prox (operator/func/norm.py:352-364),
// PositiveOrthant.prox / L1Norm.prox.
//
// Why the normal form.  The reference evaluates H^T (H yk - y): two zero-boundary separable
// correlations in sequence, i.e. four 1-D passes of 2R+1 taps whose halos compound (a fused tile
// must recompute a 2R halo of H yk).  H is separable, H = H0 (x) H1, so G = H^T H = G0 (x) G1 with
// G_a = H_a^T H_a a banded n_a x n_a matrix: in rows R <= i < n_a - R it is the Toeplitz filter
// g[d] = sum_t k[t] k[t+d], |d| <= 2R (autocorrelation of the taps); in the R boundary rows on each
// side the zero-boundary truncation of the inner H changes the coefficients, and those rows are
// evaluated exactly as sum_t k[t] [0 <= i-t < n] sum_s k[s] yk[i-t+s].  G is therefore EXACTLY the
// reference's operator (fp64 trajectories agree to 1e-16); only fp32 rounding order differs
// (measured 1.5e-7 relative after 100 PGD iterations vs fp64, the same as the reference's own fp32
// path).  Two passes of 4R+1 taps replace four passes of 2R+1, one LDS round trip and two barriers
// disappear, and b = H^T y replaces y in the compulsory traffic (x, x_prev, b in; x_new out).
//
// One 256-thread workgroup owns a TY x TX output tile:
//   phase 0  A  = yk on rows [ty0-2R, ty0+TY+2R) x cols [tx0-CA, tx0+TX+CA), zero outside the image
//   pass A   PT = (G0 yk) on the tile rows, all A columns, stored TRANSPOSED ([col][row])   (V x V
//                 register blocks: ds_read_b128 rows, packed FMAs, ds_write_b128 columns)
//   pass B   out = G1 along each row (sweeps PT rows = image columns) - b + Grad^T q, prox, store;
//                 q is evaluated on the fly from yk in A (5 x 3 stencil of yk per 4 x 2 block).
// LDS pitches / lane orders are conflict-free for R = 6 fp32 under the MI355X_MICROARCH.md §LDS
// bank model (scripts/ldsbank.py).  The blockIdx -> tile map is XCD-aware: each of the 8 XCDs owns a
// contiguous band of tiles so that halo re-reads of x / x_prev hit its own L2.
#include "tile2d.hpp"

namespace pxa {
namespace {

using namespace tile2d;


template <typename T>
struct PgdParams {
  int64_t stack, y_images;
  int n0, n1;
  int tiles0, tiles1;
  unsigned ntiles;
  T k0[2 * kMaxR + 1], k1[2 * kMaxR + 1];  // H taps, dense window t = -R..R (index t + R)
  T g0[kMaxG], g1[kMaxG];                  // interior G taps, d = -2R..2R (index d + 2R)
  T g0a, g0b, g1a, g1b;                    // forward-difference taps per axis (-1/h, 1/h)
  T lam, mu, inv_mu, a, tau, pw;
  int prox;  // 0 none, 1 positive orthant, 2 l1 (uniform branch)
  bool tv;   // lam != 0 (uniform branch)
  bool vec_ok;
  int prio;  // PXA_TUNE_PGD_PRIO mode (uniform)
};

// s_setprio with a runtime (wave-uniform) level 0..3
__device__ inline void set_prio(int lvl) {
  switch (lvl) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
  }
}

// q-weight: lam / max(|v|, mu)  (so that q = w v = lam (v - prox_{mu L21}(v)) / mu).
template <typename T>
__device__ inline T tv_weight(T n2, T lam, T mu, T inv_mu) {
  const T n = sqrt(n2);
  return lam / (n > mu ? n : mu);
}
template <>
__device__ inline float tv_weight<float>(float n2, float lam, float mu, float inv_mu) {
  const float r = __builtin_amdgcn_rsqf(n2);  // 1/|v| (inf at 0), 1 ulp
  return lam * (r < inv_mu ? r : inv_mu);
}

// ---- phase 0 of the tile kernel: yk = (x - x_prev) * a + x on the A window, zero outside the image.
// All K0 vector pairs of a thread are loaded before the first LDS store, so their latencies overlap.
struct NoHook {
  __device__ void operator()() const {}
};

template <typename T, int R, bool EDGE, typename Hook = NoHook>
__device__ inline void load_window(const PgdParams<T>& p, T* A, int ty0, int tx0, const T* __restrict__ xs,
                                   const T* __restrict__ xps, Hook&& after_issue = Hook()) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
  constexpr int CA = L::CA;
  const int n0 = p.n0, n1 = p.n1;
  const int tid = threadIdx.x;
  constexpr int K0 = cdiv(L::N0, kThreads);
  T xv[K0][V], pv[K0][V];
#pragma unroll
  for (int k = 0; k < K0; ++k) {
    const int it = tid + k * kThreads;
    if (it < L::N0) {
      const int r = it / L::NGA, g = it - r * L::NGA;
      const int gr = ty0 - 2 * R + r, gc = tx0 - CA + V * g;
      if (!EDGE) {
        const unsigned off = (unsigned)(gr * n1 + gc);
        ld_vec<T, V>(xs + off, xv[k]);
        ld_vec<T, V>(xps + off, pv[k]);
      } else if (gr >= 0 && gr < n0 && p.vec_ok && gc >= 0 && gc + V <= n1) {
        ld_vec<T, V>(xs + (int64_t)gr * n1 + gc, xv[k]);
        ld_vec<T, V>(xps + (int64_t)gr * n1 + gc, pv[k]);
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const bool in = gr >= 0 && gr < n0 && gc + v >= 0 && gc + v < n1;
          xv[k][v] = in ? xs[(int64_t)gr * n1 + gc + v] : T(0);
          pv[k][v] = in ? xps[(int64_t)gr * n1 + gc + v] : T(0);
        }
      }
    }
  }
  after_issue();  // more loads whose latency overlaps the window's (issued after it: in-order vmcnt)
#pragma unroll
  for (int k = 0; k < K0; ++k) {
    const int it = tid + k * kThreads;
    if (it < L::N0) {
      const int r = it / L::NGA, g = it - r * L::NGA;
      T out[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        T d = xv[k][v] - pv[k][v];
        d = d * p.a;
        out[v] = d + xv[k][v];
      }
      st_vec<T, V>(A + r * L::AP + V * g, out);
    }
  }
}

// ---- pass A: PT[col][row] = (G0 yk)[row][col] for the TY tile rows and all A columns
template <typename T, int R, bool EDGE>
__device__ inline void pass_a(const PgdParams<T>& p, const T* A, T* PT, const T* KT, int ty0) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
  const int tid = threadIdx.x;
  constexpr int KA = cdiv(L::NPA, kThreads);
  const bool edge_rows = EDGE && (ty0 < R || ty0 + TY > p.n0 - R);
#pragma unroll
  for (int k = 0; k < KA; ++k) {
    const int it = tid + k * kThreads;
    if (it < L::NPA) {
      const int a = it % L::NA, b = it / L::NA;  // row group fastest (conflict-free reads/writes)
      T acc[V][V];
      sweep<T, R, V, L::AP>(A + (V * a) * L::AP + V * b, p.g0, acc);
      if (edge_rows) ghost_fix<T, R, V, L::AP>(ty0 + V * a, p.n0, ty0 - 2 * R, A + V * b, p.k0, KT, acc);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        T colv[V];
#pragma unroll
        for (int u = 0; u < V; ++u) colv[u] = acc[u][v];
        st_vec<T, V>(PT + (V * b + v) * L::PTP + V * a, colv);
      }
    }
  }
}

// ---- epilogue of CW pixels of one row: z = ((G yk + Grad^T q) - b) * (-tau) + yk; prox; store;
// RelError partials sum (x_new - x)^2, sum x^2 in double.
template <typename T, int CW, bool EDGE>
__device__ inline void finish_run(const PgdParams<T>& p, int gr, int gc, const T (&g)[CW], const T (&bv)[CW],
                                  const T (&yc)[CW], const T* __restrict__ xs, T* __restrict__ xns, bool want_part,
                                  double& part_d, double& part_x) {
  const int n0 = p.n0, n1 = p.n1;
  T xo[CW];
#pragma unroll
  for (int w = 0; w < CW; ++w) {
    T gsum = g[w] - bv[w];  // (G yk + Grad^T q) - H^T y
    T z = gsum * (-p.tau);
    z = z + yc[w];
    xo[w] = apply_prox<T>(p.prox, z, p.pw);
  }
  if (!EDGE) {
    const unsigned off = (unsigned)(gr * n1 + gc);
    if constexpr (CW == 4) {
      *reinterpret_cast<float4*>(xns + off) = make_float4(xo[0], xo[1], xo[2], xo[3]);
    } else if constexpr (CW == 2 && sizeof(T) == 4) {
      *reinterpret_cast<float2*>(xns + off) = make_float2(xo[0], xo[1]);
    } else if constexpr (CW == 2) {
      st_vec<T, 2>(xns + off, xo);
    } else {
      xns[off] = xo[0];
    }
    if (want_part) {
      T xv[CW];
      if constexpr (CW * sizeof(T) == 16) ld_vec<T, CW>(xs + off, xv);
      else {
#pragma unroll
        for (int w = 0; w < CW; ++w) xv[w] = xs[off + w];
      }
#pragma unroll
      for (int w = 0; w < CW; ++w) {
        const double dd = (double)xo[w] - (double)xv[w];
        part_d += dd * dd;
        part_x += (double)xv[w] * (double)xv[w];
      }
    }
  } else if (gr < n0) {
#pragma unroll
    for (int w = 0; w < CW; ++w) {
      if (gc + w < n1) {
        xns[(int64_t)gr * n1 + gc + w] = xo[w];
        if (want_part) {
          const T xv = xs[(int64_t)gr * n1 + gc + w];
          const double dd = (double)xo[w] - (double)xv;
          part_d += dd * dd;
          part_x += (double)xv * (double)xv;
        }
      }
    }
  }
}

// ---- pass B: G1 along rows + Grad^T q, handed per output row-run to
// `emit(k, u, gr, gc, g, yc)`: g = (G yk + Grad^T q) at row gr, columns gc .. gc + CW - 1 of item k,
// yc = yk there.  The emitter finishes the pixels in place (finish_run) or stages g for the
// coalesced epilogue (epilogue_staged).
template <typename T, int R, bool EDGE, typename Emit>
__device__ inline void pass_b(const PgdParams<T>& p, const T* A, const T* PT, const T* KT, int ty0, int tx0,
                              Emit&& emit) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
  constexpr int CA = L::CA;
  constexpr int CW = L::CW;
  const int n0 = p.n0, n1 = p.n1;
  const int tid = threadIdx.x;
  constexpr int KB = cdiv(L::NPB, kThreads);
  const bool edge_cols = EDGE && (tx0 < R || tx0 + TX > n1 - R);
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    const int it = tid + k * kThreads;
    if (it < L::NPB) {
      int a, cb;
      L::pass_b_item(it, a, cb);
      const int c0 = CW * cb;  // first output column of the item (tile-relative)
      // yk window rows V a - 1 .. V a + V, cols c0 - 1 .. c0 + CW, streamed two rows at a time so
      // that the TV stencil keeps ~20 values live instead of the whole (V+2) x (CW+2) window
      auto yrow = [&](int r, T(&y)[CW + 2]) {
        const T* arow = A + (V * a - 1 + r + 2 * R) * L::AP + CA + c0;
        if constexpr (CW == 2) {
          T lo[2], mid[2], hi[2];
          ld_pair<T>(arow - 2, lo);
          ld_pair<T>(arow, mid);
          ld_pair<T>(arow + 2, hi);
          y[0] = lo[1];
          y[1] = mid[0];
          y[2] = mid[1];
          y[3] = hi[0];
        } else {
#pragma unroll
          for (int c = 0; c < CW + 2; ++c) y[c] = arow[c - 1];
        }
      };
      // q = w v at window row r (0..V), cols c = 0..CW, from yk rows r (yr) and r + 1 (yn)
      auto qrow = [&](int r, const T(&yr)[CW + 2], const T(&yn)[CW + 2], T(&q0)[CW + 1], T(&q1)[CW + 1]) {
#pragma unroll
        for (int c = 0; c <= CW; ++c) {
          const T v0 = p.g0a * yr[c] + p.g0b * yn[c];
          const T v1 = p.g1a * yr[c] + p.g1b * yr[c + 1];
          T w = tv_weight<T>(v0 * v0 + v1 * v1, p.lam, p.mu, p.inv_mu);
          if (EDGE) {
            const int gr = ty0 + V * a - 1 + r, gc = tx0 + c0 - 1 + c;
            if (!(gr >= 0 && gr < n0 && gc >= 0 && gc < n1)) w = T(0);
          }
          q0[c] = v0 * w;
          q1[c] = v1 * w;
        }
      };
      T yc[V][CW];  // yk at the item's own pixels
      T tv[V][CW];
      {
        T yr[CW + 2], yn[CW + 2];
        yrow(0, yr);
        yrow(1, yn);
        T qp0[CW + 1], qp1[CW + 1];
        if (p.tv) qrow(0, yr, yn, qp0, qp1);
#pragma unroll
        for (int u = 0; u < V; ++u) {
#pragma unroll
          for (int c = 0; c < CW + 2; ++c) yr[c] = yn[c];  // window row u + 1
          yrow(u + 2, yn);
#pragma unroll
          for (int w = 0; w < CW; ++w) yc[u][w] = yr[w + 1];
          if (p.tv) {
            T qc0[CW + 1], qc1[CW + 1];
            qrow(u + 1, yr, yn, qc0, qc1);
            // Grad^T q: flipped 2-tap adjoints, (+1/h tap at i - e_d) then (-1/h tap at i), summed over d
#pragma unroll
            for (int w = 0; w < CW; ++w) {
              const T t0 = p.g0b * qp0[w + 1] + p.g0a * qc0[w + 1];
              const T t1 = p.g1b * qc1[w] + p.g1a * qc1[w + 1];
              tv[u][w] = t0 + t1;
            }
#pragma unroll
            for (int c = 0; c <= CW; ++c) qp0[c] = qc0[c];
          }
        }
      }
      T acc[CW][V];            // acc[w][u]: column c0 + w, row V a + u
      sweep<T, R, CW, L::PTP>(PT + (CA - 2 * R + c0) * L::PTP + V * a, p.g1, acc);
      if (edge_cols) ghost_fix<T, R, CW, L::PTP>(tx0 + c0, n1, tx0 - CA, PT + V * a, p.k1, KT + kKT, acc);
#pragma unroll
      for (int u = 0; u < V; ++u) {
        T g[CW], y[CW];
#pragma unroll
        for (int w = 0; w < CW; ++w) {
          g[w] = p.tv ? acc[w][u] + tv[u][w] : acc[w][u];
          y[w] = yc[u][w];
        }
        emit(k, u, ty0 + V * a + u, tx0 + c0, g, y);
      }
    }
  }
}

// ---- staged epilogue: every thread parks g = G yk + Grad^T q of its pass-B pixels in O (the PT
// region, free once all G1 sweeps are done), then the workgroup finishes the tile in row-major order:
// each 16-B vector of a row is one lane (16 lanes per fp32 row), so H^T y / x loads and x_new stores
// are full 128-B lines instead of the pass-B item order's 64-B row pieces (measured on MI355X: a
// 2048^2 fp32 store in the item order 7.2 us, row-major 5.2 us).  yk comes from A.
template <typename T, int R, bool EDGE>
__device__ inline void epilogue_staged(const PgdParams<T>& p, const T* A, const T* O, int ty0, int tx0,
                                       const T* __restrict__ bs, const T* __restrict__ xs, T* __restrict__ xns,
                                       bool want_part, double& part_d, double& part_x) {
  using L = Layout<T, R>;
  using S = Stage<T, R>;
  constexpr int V = L::V;
  const int n0 = p.n0, n1 = p.n1;
  int r0, cq;
  S::lane(threadIdx.x, r0, cq);
  constexpr int NS = TY / S::RPS;
  T bv[NS][V];
#pragma unroll
  for (int s = 0; s < NS; ++s) {  // all H^T y loads first: one round trip
    const int gr = ty0 + r0 + s * S::RPS, gc = tx0 + V * cq;
    if (!EDGE) {
      ld_vec<T, V>(bs + (unsigned)(gr * n1 + gc), bv[s]);
    } else {
#pragma unroll
      for (int v = 0; v < V; ++v) bv[s][v] = (gr < n0 && gc + v < n1) ? bs[(int64_t)gr * n1 + gc + v] : T(0);
    }
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int r = r0 + s * S::RPS;
    T g[V], y[V];
    ld_vec<T, V>(O + S::idx(r, V * cq), g);
    ld_vec<T, V>(A + (r + 2 * R) * L::AP + L::CA + V * cq, y);
    finish_run<T, V, EDGE>(p, ty0 + r, tx0 + V * cq, g, bv[s], y, xs, xns, want_part, part_d, part_x);
  }
}

// Workgroup fold of the per-thread RelError partials into partials[2 tile .. 2 tile + 1] (fixed order).
// `red`: 2 * kThreads / 64 doubles of LDS that no other phase touches between the two barriers.
template <typename Barrier>
__device__ inline void fold_partials(double part_d, double part_x, double* red, double* partials, unsigned tile,
                                     Barrier&& barrier) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    part_d += __shfl_down(part_d, off, 64);
    part_x += __shfl_down(part_x, off, 64);
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  barrier();
  if (lane == 0) {
    red[w] = part_d;
    red[kThreads / 64 + w] = part_x;
  }
  barrier();
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

// H^T y at row gr, columns gc .. gc + CW - 1 (zero outside the image on edge tiles)
template <typename T, int CW, bool EDGE>
__device__ inline void load_b(const T* __restrict__ bs, int gr, int gc, int n0, int n1, T (&bv)[CW]) {
  if (!EDGE) {
    if constexpr (CW == 2) ld_pair<T>(bs + (unsigned)(gr * n1 + gc), bv);
    else bv[0] = bs[(unsigned)(gr * n1 + gc)];
  } else {
#pragma unroll
    for (int w = 0; w < CW; ++w) bv[w] = (gr < n0 && gc + w < n1) ? bs[(int64_t)gr * n1 + gc + w] : T(0);
  }
}

// STAGED (the default): pass B parks its results in LDS and the tile is finished in row-major order
// (epilogue_staged); otherwise each pass-B item finishes its own pixels (finish_run in item order).
template <typename T, int R, bool EDGE, bool STAGED>
__device__ inline void pgd_tile(const PgdParams<T>& p, unsigned char* smem, unsigned tile, int ty0, int tx0,
                                const T* __restrict__ xs, const T* __restrict__ xps, const T* __restrict__ bs,
                                T* __restrict__ xns, double* __restrict__ partials) {
  using L = Layout<T, R>;
  constexpr int CW = L::CW;
  constexpr int V = L::V;
  constexpr int KB = cdiv(L::NPB, kThreads);
  T* A = reinterpret_cast<T*>(smem);
  T* PT = A + L::AR * L::AP;
  T* KT = PT + L::AC * L::PTP;  // H taps for runtime-indexed reads (boundary corrections)
  const int n0 = p.n0, n1 = p.n1;
  const int tid = threadIdx.x;
  if (EDGE && tid < 2 * R + 1) {
    KT[tid] = p.k0[tid];
    KT[kKT + tid] = p.k1[tid];
  }
  double part_d = 0.0, part_x = 0.0;
  const int pm = p.prio;
  const int base_prio = pm == 1 || pm == 4 ? (int)((blockIdx.x >> 8) & 3u) : pm == 3 ? (int)((blockIdx.x >> 3) & 3u) : 0;
  const bool phase_prio = pm == 2 || pm == 4;
  if (pm) set_prio(phase_prio ? 3 : base_prio);
  if constexpr (STAGED) {
    using S = Stage<T, R>;
    load_window<T, R, EDGE>(p, A, ty0, tx0, xs, xps);
    if (phase_prio) set_prio(base_prio);
    __syncthreads();
    pass_a<T, R, EDGE>(p, A, PT, KT, ty0);
    __syncthreads();
    T st[KB][V][CW];
    pass_b<T, R, EDGE>(p, A, PT, KT, ty0, tx0, [&](int k, int u, int, int, const T(&g)[CW], const T(&)[CW]) {
#pragma unroll
      for (int w = 0; w < CW; ++w) st[k][u][w] = g[w];
    });
    __syncthreads();  // every G1 sweep is done with PT: O may overwrite it
    T* O = PT;
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int it = tid + k * kThreads;
      if (it < L::NPB) {
        int a, cb;
        L::pass_b_item(it, a, cb);
#pragma unroll
        for (int u = 0; u < V; ++u) {
          T* o = O + S::idx(V * a + u, CW * cb);
          if constexpr (CW == 2) {
            const T pr[2] = {st[k][u][0], st[k][u][1]};
            if constexpr (sizeof(T) == 4) *reinterpret_cast<float2*>(o) = make_float2(pr[0], pr[1]);
            else st_vec<T, 2>(o, pr);
          } else {
            o[0] = st[k][u][0];
          }
        }
      }
    }
    __syncthreads();
    if (phase_prio) set_prio(3);
    epilogue_staged<T, R, EDGE>(p, A, O, ty0, tx0, bs, xs, xns, partials != nullptr, part_d, part_x);
    if (partials) fold_partials(part_d, part_x, reinterpret_cast<double*>(smem), partials, tile, [] { __syncthreads(); });
  } else {
    load_window<T, R, EDGE>(p, A, ty0, tx0, xs, xps);
    __syncthreads();
    pass_a<T, R, EDGE>(p, A, PT, KT, ty0);
    __syncthreads();
    const bool want = partials != nullptr;
    pass_b<T, R, EDGE>(p, A, PT, KT, ty0, tx0, [&](int, int, int gr, int gc, const T(&g)[CW], const T(&y)[CW]) {
      T bv[CW];
      load_b<T, CW, EDGE>(bs, gr, gc, n0, n1, bv);
      finish_run<T, CW, EDGE>(p, gr, gc, g, bv, y, xs, xns, want, part_d, part_x);
    });
    if (partials) {
      // A / PT are free again once every thread is past pass B
      fold_partials(part_d, part_x, reinterpret_cast<double*>(smem), partials, tile, [] { __syncthreads(); });
    }
  }
}

template <typename T, int R, bool STAGED>
__global__ void __launch_bounds__(kThreads, 4) pgd_tv2d_kernel(PgdParams<T> p, const T* __restrict__ x,
                                                            const T* __restrict__ xp, const T* __restrict__ b,
                                                            T* __restrict__ xn, double* __restrict__ partials) {
  using L = Layout<T, R>;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const unsigned tile = xcd_tile(blockIdx.x, p.ntiles);
  const unsigned tpi = (unsigned)p.tiles0 * (unsigned)p.tiles1;
  const unsigned s = tile / tpi;
  const unsigned tr = tile - s * tpi;
  const unsigned trow = tr / (unsigned)p.tiles1;
  const int ty0 = (int)trow * TY, tx0 = (int)(tr - trow * (unsigned)p.tiles1) * TX;
  const int64_t img = (int64_t)p.n0 * p.n1;
  const T* xs = x + (int64_t)s * img;
  const T* xps = xp + (int64_t)s * img;
  const T* bs = b + (int64_t)(s % (unsigned)p.y_images) * img;
  T* xns = xn + (int64_t)s * img;
  // interior: the whole A window lies inside the image (so no boundary rows / columns of G either),
  // rows are 16-B aligned and 32-bit offsets suffice -> no bounds tests
  const bool interior = p.vec_ok && img <= 0x7fffffff && ty0 - 2 * R >= 0 && ty0 + TY + 2 * R <= p.n0 &&
                        tx0 - L::CA >= 0 && tx0 + TX + L::CA <= p.n1;
  if (interior)
    pgd_tile<T, R, false, STAGED>(p, smem_raw, tile, ty0, tx0, xs, xps, bs, xns, partials);
  else
    pgd_tile<T, R, true, STAGED>(p, smem_raw, tile, ty0, tx0, xs, xps, bs, xns, partials);
}

template <typename T, int R, bool STAGED>
int launch_pgd_v(const PgdParams<T>& p, const void* x, const void* xp, const void* b, void* xn, double* partials,
                 hipStream_t s) {
  using L = Layout<T, R>;
  const size_t smem = L::BYTES;
  auto kern = pgd_tv2d_kernel<T, R, STAGED>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(p.ntiles), dim3(kThreads), smem, s, p, (const T*)x, (const T*)xp, (const T*)b,
                     (T*)xn, partials);
  return last_launch_status();
}

template <typename T, int R>
int launch_pgd(const PgdParams<T>& p, const void* x, const void* xp, const void* b, void* xn, double* partials,
               hipStream_t s) {
  // 4: item-order epilogue (the round-1 kernel), kept selectable for A/B measurements
  if (tuning(PXA_TUNE_PGD_KERNEL) == 4) return launch_pgd_v<T, R, false>(p, x, xp, b, xn, partials, s);
  return launch_pgd_v<T, R, true>(p, x, xp, b, xn, partials, s);
}

// =====================================================================================================
// Persistent LDS-DMA pipelined form (fp32, n1 % 4 == 0, 16-B aligned arrays): the same per-tile
// arithmetic (load_window's yk, pass_a, pass_b), with the global->on-chip traffic of tile t+1 in
// flight while tile t computes.
//
// The tile kernel above serialises, per workgroup, window load -> pass A -> pass B (with H^T y loads
// in its epilogue), and its 2 048 workgroups run as two synchronous rounds of 4 per CU: HBM idles
// while every CU computes (SQ_WAIT_ANY ~50 % of wave cycles, r02a profiles).  Here 2 workgroups per
// CU loop over their tiles (XCD-banded order):
//   top:    own LDS-DMA of x / x_prev windows(t) landed (counted vmcnt) -> barrier
//           issue H^T y(t) loads into registers (inline asm: counted by hand, see below)
//           convert raw windows S -> yk in A (the tile kernel's phase-0 arithmetic)   -> barrier
//           issue LDS-DMA of the x / x_prev windows of tile t+1 into S (global_load_lds_dwordx4)
//           pass A (A -> PT)                                                         -> barrier
//           vmcnt(NDW): H^T y(t) registers landed, tile t+1's DMA may stay in flight
//           pass B (PT, A, H^T y regs -> x_new)
// hipcc waits vmcnt(0) at the first use of an ordinary global load while an LDS-DMA is in flight
// (cdna_hip_programming.md §5 "Pipelining across barriers"), which would drain tile t+1's DMA before
// pass B: the H^T y loads are inline-asm global_load_dwordx2 with a hand-counted wait instead, and
// barriers are raw s_barrier (a __syncthreads() would also drain the DMA).  Out-of-image window
// slots DMA from a 16-byte zero page.  Each wave issues exactly NDW DMA instructions per tile (the
// surplus instruction of the last wave and the tail window re-write slots with identical bytes), so
// the hand-counted vmcnt values are exact.
__device__ __attribute__((aligned(16))) float g_zero_page[4];

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

template <int R>
struct V5 {
  using L = Layout<float, R>;
  static constexpr int SV = L::AC / 4;             // 16-B vectors per staged window row (unpadded)
  static constexpr int SSLOTS = L::AR * SV;        // vectors per staged array
  static constexpr int NSLOT = 2 * SSLOTS;         // x window then x_prev window
  static constexpr int NDMA = cdiv(NSLOT, 64);     // wave-instructions per tile
  static constexpr int NDW = cdiv(NDMA, kThreads / 64);  // per wave
  static constexpr int A_OFF = NSLOT * 4;          // floats
  static constexpr int PT_OFF = A_OFF + L::AR * L::AP;
  static constexpr int KT_OFF = PT_OFF + L::AC * L::PTP;
  static constexpr int RED_OFF = KT_OFF + 2 * kKT; // 2 * 4 doubles
  static constexpr size_t BYTES = (size_t)(RED_OFF + 2 * 2 * (kThreads / 64)) * 4;
  static_assert(NSLOT >= 64, "window smaller than one DMA instruction");
  static_assert(NDW <= 15, "hand-counted vmcnt must fit the 6-bit counter with the b loads");
  static_assert((A_OFF % 4) == 0 && (PT_OFF % 4) == 0 && (RED_OFF % 2) == 0, "LDS carve alignment");
};

__device__ inline void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int N>
__device__ inline void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// One wave-instruction of LDS-DMA: 64 lanes x 16 B from per-lane global addresses into the
// contiguous 1 KiB at `lds_dst` (wave-uniform, passed in M0).  Written as inline asm so that hipcc
// does not see an LDS-DMA in flight: it would otherwise wait vmcnt(0) before every LDS access of
// passes A / B (it cannot tell that they touch other LDS bytes) and drain the prefetch.  All waits
// for these loads are the hand-counted ones of the persistent loop.
__device__ inline void dma16(const float* gsrc, float* lds_dst) {
  const unsigned lds_addr = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)((lds_void*)lds_dst));
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_addr)
      : "memory");
}

// this wave's NDW LDS-DMA instructions for the raw x / x_prev windows of the tile at (ty0, tx0)
template <int R, bool EDGE>
__device__ inline void issue_windows(float* S, const float* xs, const float* xps, int ty0, int tx0, int n0, int n1) {
  using P = V5<R>;
  constexpr int CA = P::L::CA;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int i = 0; i < P::NDW; ++i) {
    int ins = wave + (kThreads / 64) * i;
    if (ins > P::NDMA - 1) ins = P::NDMA - 1;  // surplus: repeat the last instruction (same bytes)
    int base = ins * 64;
    if (base > P::NSLOT - 64) base = P::NSLOT - 64;  // tail window ends at the last slot
    const int s = base + lane;
    const int arr = s >= P::SSLOTS;
    const int q = s - arr * P::SSLOTS;
    const int r = q / P::SV, g = q - r * P::SV;
    const int gr = ty0 - 2 * R + r, gc = tx0 - CA + 4 * g;
    const float* img = arr ? xps : xs;
    const float* src;
    if (!EDGE) {
      src = img + (unsigned)(gr * n1 + gc);
    } else {
      const bool in = gr >= 0 && gr < n0 && gc >= 0 && gc < n1;
      src = in ? img + (int64_t)gr * n1 + gc : g_zero_page;
    }
    dma16(src, S + 4 * base);
  }
}

__device__ inline void asm_load_b2(float2& v, const float* ptr) {
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(ptr) : "memory");
}

template <int R, bool EDGE>
__device__ inline void issue_b(float2 (&bq)[4], const float* bs, int ty0, int tx0, int n0, int n1) {
  using L = Layout<float, R>;
  int a, cb;
  L::pass_b_item(threadIdx.x, a, cb);
  const int gc = tx0 + 2 * cb;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int gr = ty0 + 4 * a + u;
    const float* ptr;
    if (!EDGE) ptr = bs + (unsigned)(gr * n1 + gc);
    else ptr = (gr < n0 && gc < n1) ? bs + (int64_t)gr * n1 + gc : g_zero_page;  // n1 even: gc < n1 => gc+1 < n1
    asm_load_b2(bq[u], ptr);
  }
}

// raw windows -> yk in A (bit-identical to load_window's arithmetic; zero page => yk = 0 outside)
template <int R>
__device__ inline void convert_windows(const float* S, float* A, float a) {
  using P = V5<R>;
  using L = typename P::L;
  const float* Sa = static_cast<const float*>(__builtin_assume_aligned(S, 16));
  float* Aa = static_cast<float*>(__builtin_assume_aligned(A, 16));
#pragma unroll
  for (int k = 0; k < cdiv(P::SSLOTS, kThreads); ++k) {
    const int it = threadIdx.x + k * kThreads;
    if (it >= P::SSLOTS) break;
    const int r = it / P::SV, g = it - r * P::SV;
    float xv[4], pv[4], out[4];
    ld_vec<float, 4>(Sa + 4 * it, xv);
    ld_vec<float, 4>(Sa + 4 * (P::SSLOTS + it), pv);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      float d = xv[v] - pv[v];
      d = d * a;
      out[v] = d + xv[v];
    }
    st_vec<float, 4>(Aa + r * L::AP + 4 * g, out);
  }
}

struct TileOf {
  unsigned tile, s;
  int ty0, tx0;
};

template <int R>
__global__ void __launch_bounds__(kThreads, 2) pgd_tv2d_persistent(PgdParams<float> p, const float* __restrict__ x,
                                                                 const float* __restrict__ xp,
                                                                 const float* __restrict__ b, float* __restrict__ xn,
                                                                 double* __restrict__ partials) {
  using P = V5<R>;
  using L = typename P::L;
  extern __shared__ __attribute__((aligned(16))) float smem5[];
  float* S = smem5;
  float* A = smem5 + P::A_OFF;
  float* PT = smem5 + P::PT_OFF;
  float* KT = smem5 + P::KT_OFF;
  double* red = reinterpret_cast<double*>(smem5 + P::RED_OFF);
  const int tid = threadIdx.x;
  const int n0 = p.n0, n1 = p.n1;
  const int64_t img = (int64_t)n0 * n1;
  const unsigned tpi = (unsigned)p.tiles0 * (unsigned)p.tiles1;
  // XCD-banded tile order: workgroup group g8 = blockIdx % 8 owns a contiguous band of tiles and its
  // G/8 workgroups sweep that band together (halo re-reads of neighbouring tiles hit the XCD's L2)
  const unsigned G8 = gridDim.x >> 3, g8 = blockIdx.x & 7u, j = blockIdx.x >> 3;
  const unsigned q8 = p.ntiles >> 3, r8 = p.ntiles & 7u;
  const unsigned band_lo = g8 * q8 + (g8 < r8 ? g8 : r8);
  const unsigned band_hi = band_lo + q8 + (g8 < r8 ? 1u : 0u);
  auto tile_at = [&](unsigned t) {
    TileOf o;
    o.tile = t;
    o.s = t / tpi;
    const unsigned tr = t - o.s * tpi;
    const unsigned trow = tr / (unsigned)p.tiles1;
    o.ty0 = (int)trow * TY;
    o.tx0 = (int)(tr - trow * (unsigned)p.tiles1) * TX;
    return o;
  };
  auto interior_at = [&](const TileOf& o) {
    return o.ty0 - 2 * R >= 0 && o.ty0 + TY + 2 * R <= n0 && o.tx0 - L::CA >= 0 && o.tx0 + TX + L::CA <= n1;
  };
  auto issue_tile = [&](const TileOf& o) {
    const float* xs = x + (int64_t)o.s * img;
    const float* xps = xp + (int64_t)o.s * img;
    if (interior_at(o)) issue_windows<R, false>(S, xs, xps, o.ty0, o.tx0, n0, n1);
    else issue_windows<R, true>(S, xs, xps, o.ty0, o.tx0, n0, n1);
  };
  if (tid < 2 * R + 1) {
    KT[tid] = p.k0[tid];
    KT[kKT + tid] = p.k1[tid];
  }
  unsigned t = band_lo + j;
  if (t < band_hi) issue_tile(tile_at(t));
  bool prev_interior = false;  // stores of the previous tile: a known count only for interior tiles
  const PgdParams<float>* pp = &p;
  for (; t < band_hi; t += G8) {
    // re-read the solver constants (taps, lam, tau, ...) from the kernel-argument segment in every
    // iteration: hoisted out of the loop they would pin ~100 SGPRs and spill to VGPR lanes
    asm volatile("" : "+s"(pp));
    const PgdParams<float>& q = *pp;
    const TileOf o = tile_at(t);
    const bool interior = interior_at(o);
    const unsigned tn = t + G8;
    const bool has_next = tn < band_hi;
    // 1. this wave's DMA of tile t landed (only the previous tile's 4 x_new stores may stay in flight)
    if (prev_interior) wait_vm<4>();
    else wait_vm<0>();
    lds_barrier();  // every wave's DMA landed; the previous pass B is done with A / PT / red
    const float* xs = x + (int64_t)o.s * img;
    const float* bs = b + (int64_t)(o.s % (unsigned)p.y_images) * img;
    float* xns = xn + (int64_t)o.s * img;
    // 2. H^T y of this tile into registers (4 x dwordx2 per thread), counted by hand
    float2 bq[4];
    if (interior) issue_b<R, false>(bq, bs, o.ty0, o.tx0, n0, n1);
    else issue_b<R, true>(bq, bs, o.ty0, o.tx0, n0, n1);
    // 3. raw windows -> yk
    convert_windows<R>(S, A, q.a);
    lds_barrier();  // A complete; S free
    // 4. next tile's windows in flight during passes A and B
    if (has_next) issue_tile(tile_at(tn));
    double part_d = 0.0, part_x = 0.0;
    if (interior) {
      pass_a<float, R, false>(q, A, PT, KT, o.ty0);
      lds_barrier();
      if (has_next) wait_vm<P::NDW>();
      else wait_vm<0>();
      asm volatile("" : "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]));
      const bool want = partials != nullptr;
      pass_b<float, R, false>(q, A, PT, KT, o.ty0, o.tx0,
                           [&](int, int u, int gr, int gc, const float(&g)[2], const float(&y)[2]) {
                             const float bv[2] = {bq[u].x, bq[u].y};
                             finish_run<float, 2, false>(q, gr, gc, g, bv, y, xs, xns, want, part_d, part_x);
                           });
    } else {
      pass_a<float, R, true>(q, A, PT, KT, o.ty0);
      lds_barrier();
      if (has_next) wait_vm<P::NDW>();
      else wait_vm<0>();
      asm volatile("" : "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]));
      const bool want = partials != nullptr;
      pass_b<float, R, true>(q, A, PT, KT, o.ty0, o.tx0,
                           [&](int, int u, int gr, int gc, const float(&g)[2], const float(&y)[2]) {
                             const float bv[2] = {bq[u].x, bq[u].y};
                             finish_run<float, 2, true>(q, gr, gc, g, bv, y, xs, xns, want, part_d, part_x);
                           });
    }
    if (partials) fold_partials(part_d, part_x, red, partials, o.tile, [] { lds_barrier(); });
    prev_interior = interior && partials == nullptr;
  }
}

template <int R>
int launch_pgd_persistent(const PgdParams<float>& p, const void* x, const void* xp, const void* b, void* xn,
                          double* partials, hipStream_t s) {
  using P = V5<R>;
  auto kern = pgd_tv2d_persistent<R>;
  static int grid_cap = 0;  // resident workgroups on this device (2 per CU by LDS), multiple of 8
  if (grid_cap == 0) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)P::BYTES);
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess) return PXA_ERR_UNSUPPORTED;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return PXA_ERR_UNSUPPORTED;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)kern, kThreads, P::BYTES) != hipSuccess)
      return PXA_ERR_UNSUPPORTED;
    if (per < 1) per = 1;
    if (per > 2) per = 2;
    grid_cap = cus * per;
  }
  int grid = grid_cap;
  if ((int64_t)grid > (int64_t)p.ntiles) grid = (int)p.ntiles;
  grid = grid < 8 ? 8 : (grid & ~7);  // the XCD banding needs a multiple of 8 (idle groups just exit)
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), P::BYTES, s, p, (const float*)x, (const float*)xp,
                     (const float*)b, (float*)xn, partials);
  return last_launch_status();
}

template <typename T>
int pgd_entry(int64_t stack, int64_t y_images, int64_t n0, int64_t n1, int nt0, const int32_t* off0,
              const double* coef0, int nt1, const int32_t* off1, const double* coef1, double h0, double h1, double lam,
              double mu, double a, double tau, int prox, double prox_w, const void* x, const void* x_prev,
              const void* hty, void* x_new, double* partials, hipStream_t s) {
  PXA_CHECK_ARG(stack >= 1 && n0 >= 1 && n1 >= 1 && y_images >= 1 && stack % y_images == 0);
  PXA_CHECK_ARG(n0 <= 0x7fffffff && n1 <= 0x7fffffff);
  PXA_CHECK_ARG(x && x_prev && hty && x_new);
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
  p.n0 = (int)n0;
  p.n1 = (int)n1;
  p.tiles0 = (int)((n0 + TY - 1) / TY);
  p.tiles1 = (int)((n1 + TX - 1) / TX);
  const int64_t ntiles = stack * (int64_t)p.tiles0 * p.tiles1;
  PXA_CHECK_ARG(ntiles <= 0x7fffffff);
  p.ntiles = (unsigned)ntiles;
  // H taps as a dense window in double (code-generation order folded per offset), then G = k (*) k
  double k0[2 * kMaxR + 1] = {0}, k1[2 * kMaxR + 1] = {0};
  for (int q = 0; q < nt0; ++q) k0[off0[q] + R] += coef0[q];
  for (int q = 0; q < nt1; ++q) k1[off1[q] + R] += coef1[q];
  for (int j = 0; j < 2 * kMaxR + 1; ++j) {
    p.k0[j] = (T)k0[j];
    p.k1[j] = (T)k1[j];
  }
  for (int d = -2 * R; d <= 2 * R; ++d) {
    double s0 = 0.0, s1 = 0.0;
    for (int t = -R; t <= R; ++t) {
      if (t + d < -R || t + d > R) continue;
      s0 += k0[t + R] * k0[t + d + R];
      s1 += k1[t + R] * k1[t + d + R];
    }
    p.g0[d + 2 * R] = (T)s0;
    p.g1[d + 2 * R] = (T)s1;
  }
  for (int j = 4 * R + 1; j < kMaxG; ++j) p.g0[j] = p.g1[j] = T(0);
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
  p.vec_ok = (n1 % V == 0) && aligned16(x) && aligned16(x_prev) && aligned16(hty) && aligned16(x_new);
  p.tv = lam != 0.0;
  p.prox = prox;
  p.prio = tuning(PXA_TUNE_PGD_PRIO);
  if constexpr (sizeof(T) == 4) {
    // persistent LDS-DMA kernel (opt-in, PXA_TUNE_PGD_KERNEL = 5): 16-B vectors along rows and 32-bit
  // in-image offsets.  Measured slower than the tile kernel at 2048^2 (50 vs 27 us): see its header.
    if (p.vec_ok && n0 * n1 <= 0x7fffffff && tuning(PXA_TUNE_PGD_KERNEL) == 5) {
      switch (R) {
        case 1: return launch_pgd_persistent<1>(p, x, x_prev, hty, x_new, partials, s);
        case 2: return launch_pgd_persistent<2>(p, x, x_prev, hty, x_new, partials, s);
        case 3: return launch_pgd_persistent<3>(p, x, x_prev, hty, x_new, partials, s);
        case 4: return launch_pgd_persistent<4>(p, x, x_prev, hty, x_new, partials, s);
        case 5: return launch_pgd_persistent<5>(p, x, x_prev, hty, x_new, partials, s);
        case 6: return launch_pgd_persistent<6>(p, x, x_prev, hty, x_new, partials, s);
        case 7: return launch_pgd_persistent<7>(p, x, x_prev, hty, x_new, partials, s);
        default: return launch_pgd_persistent<8>(p, x, x_prev, hty, x_new, partials, s);
      }
    }
  }
  switch (R) {
    case 1: return launch_pgd<T, 1>(p, x, x_prev, hty, x_new, partials, s);
    case 2: return launch_pgd<T, 2>(p, x, x_prev, hty, x_new, partials, s);
    case 3: return launch_pgd<T, 3>(p, x, x_prev, hty, x_new, partials, s);
    case 4: return launch_pgd<T, 4>(p, x, x_prev, hty, x_new, partials, s);
    case 5: return launch_pgd<T, 5>(p, x, x_prev, hty, x_new, partials, s);
    case 6: return launch_pgd<T, 6>(p, x, x_prev, hty, x_new, partials, s);
    case 7: return launch_pgd<T, 7>(p, x, x_prev, hty, x_new, partials, s);
    default: return launch_pgd<T, 8>(p, x, x_prev, hty, x_new, partials, s);
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
                      const void* x_prev, const void* hty, void* x_new, double* partials, void* stream) {
  PXA_DISPATCH(dtype, T,
               return pgd_entry<T>(stack, y_images, n0, n1, nt0, off0, coef0, nt1, off1, coef1, h0, h1, lam, mu, a,
                                   tau, prox, prox_w, x, x_prev, hty, x_new, partials, as_stream(stream)));
}

}  // extern "C"
