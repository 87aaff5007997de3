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
  int diag;  // PXA_TUNE_PGD_DIAG (timing probes; bit 5: phase trace)
};

// Timing trace (PXA_TUNE_PGD_DIAG bit 5, read by pxa_pgd_march_trace): s_memtime stamps of waves 0-3 of
// a few workgroups.  March kernel: workgroups 0 and grid/2, 8 points of each of their first 16 bands.
// Tile kernel: workgroups 0, 1, grid/2 and grid-1, 8 points of their tile.  Staged in LDS beyond the
// kernels' own carve, dumped at exit.
constexpr int kTraceWords = 2 * 4 * 16 * 8;
__device__ unsigned long long g_march_trace[kTraceWords];

// s_setprio with a runtime (wave-uniform) level 0..3
__device__ inline void set_prio(int lvl) {
  switch (lvl) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
  }
}

// Every multiply-add outside the Toeplitz sweeps is written as an explicit fma (the TV stencil's
// two-product sums as fma(a, b, c * d)): under fp-contract=fast the compiler fuses or not, and picks
// which product to fuse, per code position, so the tile and march kernels (different blocking, code
// layout per radius) would otherwise round differently at a few pixels.
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
        out[v] = fma(xv[k][v] - pv[k][v], p.a, xv[k][v]);  // (x - x_prev) * a + x, one rounding site
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
  // one item per thread (fp32): items spread over all 4 waves in chunks of a multiple of NA, so each
  // lane keeps it % NA == lane % NA (the conflict-free lane pattern) -- e.g. 48 / 48 / 48 / 32 for the
  // 176 items of R = 6, where consecutive numbering leaves wave 3 idle through pass A
  constexpr int CH = KA == 1 ? rup(cdiv(L::NPA, kThreads / 64), L::NA) : 64;
  static_assert(KA > 1 || CH <= 64, "pass-A chunk fits a wave");
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
    T z = fma(gsum, -p.tau, yc[w]);
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
__device__ inline void pass_b(const PgdParams<T>& p, const T* A, const T* PT, const T* KT, const T* GH, int ty0, int tx0,
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
          const T v0 = fma(p.g0a, yr[c], p.g0b * yn[c]);
          const T v1 = fma(p.g1a, yr[c], p.g1b * yr[c + 1]);
          T w = tv_weight<T>(fma(v0, v0, v1 * v1), p.lam, p.mu, p.inv_mu);
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
              const T t0 = fma(p.g0b, qp0[w + 1], p.g0a * qc0[w + 1]);
              const T t1 = fma(p.g1b, qc1[w], p.g1a * qc1[w + 1]);
              tv[u][w] = t0 + t1;
            }
#pragma unroll
            for (int c = 0; c <= CW; ++c) qp0[c] = qc0[c];
          }
        }
      }
      T acc[CW][V];            // acc[w][u]: column c0 + w, row V a + u
      sweep<T, R, CW, L::PTP>(PT + (CA - 2 * R + c0) * L::PTP + V * a, p.g1, acc);
      if (edge_cols) ghost_fix_pre<T, R, CW, TY>(tx0 + c0, n1, V * a, GH, KT + kKT, acc);
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
// H^T y of this thread's staged-epilogue pixels (NS row-major 16-B vectors), zero outside the image;
// issued before the O staging so that its latency overlaps the staging and its barrier
template <typename T, int R>
struct StagedB {
  static constexpr int NS = TY / Stage<T, R>::RPS;
  T v[NS][kVecN<T>];
};

template <typename T, int R, bool EDGE>
__device__ inline void load_b_staged(const PgdParams<T>& p, int ty0, int tx0, const T* __restrict__ bs,
                                     StagedB<T, R>& b) {
  using S = Stage<T, R>;
  constexpr int V = kVecN<T>;
  const int n0 = p.n0, n1 = p.n1;
  int r0, cq;
  S::lane(threadIdx.x, r0, cq);
#pragma unroll
  for (int s = 0; s < StagedB<T, R>::NS; ++s) {  // all H^T y loads first: one round trip
    const int gr = ty0 + r0 + s * S::RPS, gc = tx0 + V * cq;
    if (!EDGE) {
      ld_vec<T, V>(bs + (unsigned)(gr * n1 + gc), b.v[s]);
    } else {
#pragma unroll
      for (int v = 0; v < V; ++v) b.v[s][v] = (gr < n0 && gc + v < n1) ? bs[(int64_t)gr * n1 + gc + v] : T(0);
    }
  }
}

template <typename T, int R, bool EDGE>
__device__ inline void epilogue_staged(const PgdParams<T>& p, const T* A, const T* O, int ty0, int tx0,
                                       const StagedB<T, R>& b, const T* __restrict__ xs, T* __restrict__ xns,
                                       bool want_part, double& part_d, double& part_x) {
  using L = Layout<T, R>;
  using S = Stage<T, R>;
  constexpr int V = L::V;
  int r0, cq;
  S::lane(threadIdx.x, r0, cq);
#pragma unroll
  for (int s = 0; s < StagedB<T, R>::NS; ++s) {
    const int r = r0 + s * S::RPS;
    T g[V], y[V];
    ld_vec<T, V>(O + S::idx(r, V * cq), g);
    ld_vec<T, V>(A + (r + 2 * R) * L::AP + L::CA + V * cq, y);
    finish_run<T, V, EDGE>(p, ty0 + r, tx0 + V * cq, g, b.v[s], y, xs, xns, want_part, part_d, part_x);
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
  T* GH = reinterpret_cast<T*>(smem + kGhOff<T, R>);  // boundary-column ghost terms (edge-column tiles)
  const int n0 = p.n0, n1 = p.n1;
  const bool edge_cols = EDGE && (tx0 < R || tx0 + TX > n1 - R);
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
  const bool tracing = (p.diag & 32) != 0;
  unsigned long long* ts = reinterpret_cast<unsigned long long*>(smem + kGhOff<T, R> + kGhBytes<T, R>);
  auto tmark = [&](int pt) {
    if (tracing && (tid & 63) == 0) ts[(tid >> 6) * 8 + pt] = clock64();
  };
  tmark(0);
  if constexpr (STAGED) {
    using S = Stage<T, R>;
    load_window<T, R, EDGE>(p, A, ty0, tx0, xs, xps);
    tmark(1);
    if (phase_prio) set_prio(base_prio);
    __syncthreads();
    tmark(2);
    pass_a<T, R, EDGE>(p, A, PT, KT, ty0);
    tmark(3);
    __syncthreads();
    if (edge_cols) {
      ghost_cols_coop<T, R>(p.k1, PT, GH, tx0, n1);
      __syncthreads();
    }
    tmark(4);
    T st[KB][V][CW];
    pass_b<T, R, EDGE>(p, A, PT, KT, GH, ty0, tx0, [&](int k, int u, int, int, const T(&g)[CW], const T(&)[CW]) {
#pragma unroll
      for (int w = 0; w < CW; ++w) st[k][u][w] = g[w];
    });
    StagedB<T, R> hb;
    load_b_staged<T, R, EDGE>(p, ty0, tx0, bs, hb);  // in flight during the O staging
    tmark(5);
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
    tmark(6);
    if (phase_prio) set_prio(3);
    epilogue_staged<T, R, EDGE>(p, A, O, ty0, tx0, hb, xs, xns, partials != nullptr, part_d, part_x);
    tmark(7);
    if (partials) fold_partials(part_d, part_x, reinterpret_cast<double*>(smem), partials, tile, [] { __syncthreads(); });
    const unsigned nb = gridDim.x, bid = blockIdx.x;
    if (tracing && (bid == 0 || bid == 1 || bid == nb / 2 || bid == nb - 1)) {
      __syncthreads();
      const int slot = bid == 0 ? 0 : bid == 1 ? 1 : bid == nb / 2 ? 2 : 3;
      if (tid < 32) g_march_trace[slot * 32 + tid] = ts[tid];
    }
  } else {
    load_window<T, R, EDGE>(p, A, ty0, tx0, xs, xps);
    __syncthreads();
    pass_a<T, R, EDGE>(p, A, PT, KT, ty0);
    __syncthreads();
    if (edge_cols) {
      ghost_cols_coop<T, R>(p.k1, PT, GH, tx0, n1);
      __syncthreads();
    }
    const bool want = partials != nullptr;
    pass_b<T, R, EDGE>(p, A, PT, KT, GH, ty0, tx0, [&](int, int, int gr, int gc, const T(&g)[CW], const T(&y)[CW]) {
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
  unsigned tile = xcd_tile(blockIdx.x, p.ntiles);
  {  // the last XCD band walks backwards: an image's bottom-edge tiles (slower: boundary corrections)
     // are dispatched first instead of last, longest-first scheduling (2048^2: 29.2-29.3 -> 28.9-29.0 us)
    const unsigned nb = p.ntiles, q8 = nb >> 3, r8 = nb & 7u, g8 = blockIdx.x & 7u;
    if (g8 == 7u) {
      const unsigned lo = 7u * q8 + (r8 < 7u ? r8 : 7u), len = q8 + (7u < r8 ? 1u : 0u);
      tile = lo + (len - 1u - (tile - lo));
    }
  }
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
  // Layout + the ghost terms (+ the timing trace under PXA_TUNE_PGD_DIAG bit 5)
  const size_t smem = kGhOff<T, R> + kGhBytes<T, R> + ((p.diag & 32) ? 256 : 0);
  auto kern = pgd_tv2d_kernel<T, R, STAGED>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(kGhOff<T, R> + kGhBytes<T, R> + 256));
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
// March kernel (fp32; R <= 6; n1 % 4 == 0; 16-B aligned arrays; no RelError partials): the tile
// kernel's per-pixel arithmetic, reorganised so that HBM traffic is in flight while the CU computes.
//
// The tile kernel serialises, per workgroup, window load -> pass A -> pass B -> epilogue, and the
// 2 048 tiles of a 2048^2 image run as two phase-locked rounds of 4 workgroups per CU: HBM idles while
// the chip computes and the VALUs idle while it loads (SQ_WAIT_ANY ~44 % of wave cycles), and every
// tile re-reads a 2R row halo above and below (the x / x_prev window is 2.4x the tile).  Here one
// workgroup owns a 64-column strip of a run of SB consecutive 16-row BANDS and marches down it:
//   * the yk window W (16 + 4R rows x the strip's 64 + 2 CA columns) is carried from band to band:
//     its last 4R rows become the next band's first 4R rows (a shift through registers), so each band
//     loads only its 16 new rows (x / x_prev read 1.375x, vertical halo once per run);
//   * those 16 new rows of x and x_prev travel by LDS-DMA (global_load_lds_dwordx4) into a staging
//     area S one band AHEAD: band k+1's rows are in flight during band k's passes A and B;
//   * H^T y of band k is loaded into registers at the top of band k and consumed by its epilogue.
// LDS per workgroup (R = 6): W 14.7 KB + S 11.3 KB + PT 8.4 KB + O 4 KB = 38.7 KB -> 4 per CU, the same
// occupancy as the tile kernel.  Per band: pass A (4 x 2 register blocks, G0 along rows, transposed
// into PT), pass B (2 x 2 blocks, G1 along PT rows + the TV stencil of yk, parked in O), and the
// staged row-major epilogue (one 16-B vector per lane: full 256-B row stores).  Every output gets the
// same fp32 operations in the same order as in the tile kernel (sweep / ghost-fix tap order, TV and
// epilogue expressions), so x_new is bit-identical (tests/test_gpu_pgd_variants.py).
//
// Hand-counted waits.  hipcc would wait vmcnt(0) at the first use of an ordinary load issued while an
// LDS-DMA is in flight, and a __syncthreads() drains all memory operations; the DMAs and the H^T y
// loads are therefore inline asm (invisible to hipcc's counter) and the barriers raw s_barrier.  Per
// wave and band, in issue order: [H^T y(k): 1 load] [DMA(k+1): NDW] [x_new(k) stores: 1 for interior
// bands, out-of-image lanes storing to a sink page].  Band k+1's top waits vmcnt(1) (DMA(k+1) landed,
// the store may stay in flight), the epilogue waits vmcnt(NDW) (H^T y landed, DMA(k+1) may stay in
// flight).  Every wave issues exactly NDW DMA instructions per band (the surplus
// instruction of the last wave repeats the last slot range with identical bytes), and out-of-image
// granules DMA from a zero page (n1 % 4 == 0: a 16-B granule is wholly inside or outside).
__device__ __attribute__((aligned(16))) float g_zero_page[4];
__device__ __attribute__((aligned(16))) float g_sink_page[4];
  // target of the march epilogue's out-of-image lanes

typedef __attribute__((address_space(3))) void lds_void;

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
// contiguous 1 KiB at `lds_dst` (wave-uniform, passed in M0).
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

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ inline void asm_load_b4(f32x4& v, const float* ptr) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(ptr) : "memory");
}

template <int R>
struct March {
  static constexpr int TB = 16;                       // band rows
  static constexpr int CA = rup(2 * R, 4);            // column halo (16-B granules)
  static constexpr int AC = TX + 2 * CA;              // window columns = PT rows
  static constexpr int SH = 4 * R;                    // window rows carried to the next band
  static constexpr int WR = TB + SH;                  // window rows
  static constexpr int AP = AC % 8 == 4 ? AC : AC + 4;  // W pitch = 4 mod 8 (see march_pass_a / _b)
  static constexpr int PTP = 24;                      // PT pitch (see march_pass_a / _b)
  static constexpr int OP = TX;                       // O rows (rotated, see oidx)
  static constexpr int SV = AC / 4;                   // 16-B granules per window row
  static constexpr int SSLOTS = TB * SV;              // granules per staged array
  static constexpr int NSLOT = 2 * SSLOTS;            // x rows then x_prev rows
  static constexpr int NDMA = cdiv(NSLOT, 64);        // wave-instructions per band
  static constexpr int NDW = cdiv(NDMA, kThreads / 64);  // per wave
  static constexpr int W_OFF = 0;
  static constexpr int S_OFF = W_OFF + WR * AP;
  static constexpr int PT_OFF = S_OFF + NSLOT * 4;
  static constexpr int O_OFF = PT_OFF + AC * PTP;
  static constexpr int KT_OFF = O_OFF + TB * OP;
  static constexpr int GH_OFF = KT_OFF + 2 * kKT;    // boundary-column ghost terms (march_ghost_cols)
  static constexpr size_t BYTES = (size_t)(GH_OFF + 2 * R * TB) * 4;
  static constexpr int NPA = (TB / 4) * (AC / 2);     // pass-A items: 4 rows x 2 columns
  static constexpr int NPB = (TB / 2) * (TX / 2);     // pass-B items: 2 rows x 2 columns
  static_assert(R >= 1 && R <= 6, "march kernel radius");
  static_assert(BYTES <= 40960, "4 workgroups per CU");
  static_assert(AC / 2 <= 48 && NPB == kThreads, "pass item maps");
  static_assert(NSLOT >= 64 && NDW <= 8, "DMA slots");
  static_assert((S_OFF % 4) == 0 && (PT_OFF % 4) == 0 && (O_OFF % 4) == 0, "16-B carve");
  // O: 64-dword rows, row r rotated by 4 (r / 2) dwords: the pass-B ds_write_b64 of 16 lanes (8 row
  // pairs x 2 column pairs) hit 32 distinct banks; a row-major epilogue lane group reads one row.
  __device__ static inline int oidx(int r, int c) { return r * OP + ((c + 4 * (r >> 1)) & (OP - 1)); }
};

// the kernel's PgdParams read in place from the kernel-argument segment (scalar loads at their uses)
using KP = const __attribute__((address_space(4))) PgdParams<float>*;

// out[o][w] = sum_{t=0}^{4R} g[t] src[(o + t) * PS + w], w = 0, 1: the tap order of sweep()
template <int R, int NO, int PS, typename GP>
__device__ inline void sweep2(const float* __restrict__ src, GP g, float (&out)[NO][2]) {
  using P = Pk<float>::type;
  P acc[NO];
#pragma unroll
  for (int o = 0; o < NO; ++o) acc[o] = Pk<float>::splat(0.0f);
#pragma unroll
  for (int j = 0; j < NO + 4 * R; ++j) {
    // volatile: keeps each row a ds_read_b64 (full LDS rate; the compiler would pair them into
    // ds_read2_b64, half rate, and bank-conflicting under the mod-32 rule of that instruction)
    const P row = *(const volatile __attribute__((address_space(3))) P*)(src + j * PS);
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      const int k = j - o;
      if (k >= 0 && k <= 4 * R) acc[o] = Pk<float>::splat(g[k]) * row + acc[o];
    }
  }
#pragma unroll
  for (int o = 0; o < NO; ++o) {
    out[o][0] = acc[o][0];
    out[o][1] = acc[o][1];
  }
}

// ghost_fix() for a 2-wide vector across the sweep axis (same terms, same order)
template <int R, int NO, int PS, typename GP>
__device__ inline void ghost_fix2(int i0, int n, int q0, const float* __restrict__ src, GP k, const float* __restrict__ kt,
                                  float (&acc)[NO][2]) {
#pragma unroll
  for (int side = 0; side < 2; ++side) {
    const int pg = side == 0 ? -R : n;
    const bool hit = side == 0 ? (i0 < R) : (i0 + NO - 1 >= n - R && i0 < n);
    if (!hit) continue;
    float gh[R][2];
#pragma unroll
    for (int m = 0; m < R; ++m) {
      const int pp = pg + m;
      gh[m][0] = gh[m][1] = 0.0f;
      if (pp >= i0 - R && pp <= i0 + NO - 1 + R) {
#pragma unroll
        for (int s = -R; s <= R; ++s) {
          const float2 w = *reinterpret_cast<const float2*>(src + (pp + s - q0) * PS);
          gh[m][0] = fma(k[s + R], w.x, gh[m][0]);
          gh[m][1] = fma(k[s + R], w.y, gh[m][1]);
        }
      }
    }
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      const int i = i0 + o;
      if (i >= n || (side == 0 ? i >= R : i < n - R)) continue;
#pragma unroll
      for (int m = 0; m < R; ++m) {
        const int t = i - (pg + m);
        if (t < -R || t > R) continue;
        const float kk = kt[t + R];
        acc[o][0] = fma(-kk, gh[m][0], acc[o][0]);
        acc[o][1] = fma(-kk, gh[m][1], acc[o][1]);
      }
    }
  }
}

// Boundary columns of pass B, computed cooperatively (edge strips only): GH[side][m][r] = sum_s k1[s]
// PT[ghost column pg + m + s][band row r], the (H1 G0 yk) values at the R zero-padded ghost columns on
// each side -- ghost_fix2's gh[m] with the same fma order.  ghost_fix2 would have the few lanes that own
// columns within R of the border compute all of them (one 13-tap sum per ghost column per lane), which
// held one wave ~6 500 cycles per band while the others waited at the next barrier.
template <int R, typename PP>
__device__ inline void march_ghost_cols(PP p, const float* PT, float* GH, int tx0, int n1) {
  using M = March<R>;
  const int t = threadIdx.x;
  if (t < 2 * R * M::TB) {
    const int side = t / (R * M::TB), m = (t / M::TB) % R, r = t % M::TB;
    const int row = (side == 0 ? -R : n1) + m - (tx0 - M::CA);  // PT row of the ghost column
    float g = 0.0f;
    if (row - R >= 0 && row + R < M::AC) {  // else no output of this strip uses it
#pragma unroll
      for (int q = -R; q <= R; ++q) g = fma(p->k1[q + R], PT[(row + q) * M::PTP + r], g);
    }
    GH[(side * R + m) * M::TB + r] = g;
  }
}

// ghost_fix2's correction step for pass B with the ghost terms read from GH (same terms, same order)
template <int R, int NO>
__device__ inline void ghost_cols_fix(int i0, int n, int rr, const float* __restrict__ GH, const float* __restrict__ kt,
                                      float (&acc)[NO][2]) {
  using M = March<R>;
#pragma unroll
  for (int side = 0; side < 2; ++side) {
    const int pg = side == 0 ? -R : n;
    const bool hit = side == 0 ? (i0 < R) : (i0 + NO - 1 >= n - R && i0 < n);
    if (!hit) continue;
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      const int i = i0 + o;
      if (i >= n || (side == 0 ? i >= R : i < n - R)) continue;
#pragma unroll
      for (int m = 0; m < R; ++m) {
        const int t = i - (pg + m);
        if (t < -R || t > R) continue;
        const float kk = kt[t + R];
        const float2 gh = *reinterpret_cast<const float2*>(GH + (side * R + m) * M::TB + rr);
        acc[o][0] = fma(-kk, gh.x, acc[o][0]);
        acc[o][1] = fma(-kk, gh.y, acc[o][1]);
      }
    }
  }
}

// this wave's NDW LDS-DMA instructions: x / x_prev rows row0 .. row0 + TB - 1 of the strip -> S
template <int R, bool EDGE>
__device__ inline void march_issue(float* S, const float* xs, const float* xps, int row0, int tx0, int n0, int n1) {
  using M = March<R>;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int i = 0; i < M::NDW; ++i) {
    int ins = wave + (kThreads / 64) * i;
    if (ins > M::NDMA - 1) ins = M::NDMA - 1;
    int base = ins * 64;
    if (base > M::NSLOT - 64) base = M::NSLOT - 64;
    const int s = base + lane;
    const int arr = s >= M::SSLOTS;
    const int q = s - arr * M::SSLOTS;
    const int r = q / M::SV, g = q - r * M::SV;
    const int gr = row0 + r, gc = tx0 - M::CA + 4 * g;
    const float* img = arr ? xps : xs;
    const float* src;
    if (!EDGE) {
      src = img + (unsigned)(gr * n1 + gc);
    } else {
      const bool in = gr >= 0 && gr < n0 && gc >= 0 && gc < n1;
      src = in ? img + (unsigned)(gr * n1 + gc) : g_zero_page;
    }
    dma16(src, S + 4 * base);
  }
}

// pass A of one band: PT[c][r] = (G0 yk)[r0 + r][c] for the 16 band rows and all AC window columns
template <int R, bool EDGE, typename PP>
__device__ inline void march_pass_a(PP p, const float* W, float* PT, const float* KT, int r0) {
  using M = March<R>;
  // lane -> (row group a = lane & 3, column pair b): 11 column pairs per wave.  A 32-lane ds_read_b64
  // group spans a = 0..3 x 8 consecutive b: rows 4 AP = 16 or 48 mod 64 dwords apart, conflict-free; an
  // 8-lane ds_write_b128 group a = 0..3 x 2 consecutive b: PT columns 2 PTP = 16 mod 32 apart, conflict-free
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int a = l & 3, q = l >> 2, b = 11 * w + q;  // rows 4a .. 4a+3, columns 2b, 2b+1
  if (q < 11 && b < M::AC / 2) {
    float acc[4][2];
    sweep2<R, 4, M::AP>(W + (4 * a) * M::AP + 2 * b, p->g0, acc);
    const int n0 = p->n0;
    const bool edge_rows = EDGE && (r0 < R || r0 + M::TB > n0 - R);
    if (edge_rows) ghost_fix2<R, 4, M::AP>(r0 + 4 * a, n0, r0 - 2 * R, W + 2 * b, p->k0, KT, acc);
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      const float colv[4] = {acc[0][w], acc[1][w], acc[2][w], acc[3][w]};
      st_vec<float, 4>(PT + (2 * b + w) * M::PTP + 4 * a, colv);
    }
  }
}

// pass B of one band: g = G1 (PT rows) + Grad^T q at 2 x 2 pixels per thread, parked in O
template <int R, bool EDGE, typename PP>
__device__ inline void march_pass_b(PP p, const float* W, const float* PT, const float* KT, float* O, int r0,
                                    int tx0, bool tv_on = true) {
  using M = March<R>;
  constexpr int CA = M::CA;
  const int n0 = p->n0, n1 = p->n1;
  // lane -> (row pair i = lane & 7, column pair j): a 32-lane ds_read_b64 group spans i = 0..7 x 4
  // consecutive j.  PT reads: columns 2 PTP = 48 mod 64 dwords apart -> 16-dword blocks, conflict-free;
  // TV reads of W (full 8-B pairs): row pairs 2 AP = 8 x odd mod 64 apart -> conflict-free; O writes:
  // rows rotated by 4 (r / 2) -> conflict-free
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int i = l & 7, j = 8 * w + (l >> 3);  // band rows 2i, 2i+1; strip columns 2j, 2j+1
  const int c0 = 2 * j;
  auto yrow = [&](int r, float(&y)[4]) {  // yk at band row 2i - 1 + r, strip columns c0 - 1 .. c0 + 2
    // three full 8-B pairs (volatile: the compiler would shrink the outer two to ds_read_b32, which
    // bank-conflict 2-way under the mod-32 rule of 4-B reads)
    using P = Pk<float>::type;
    using LP = const volatile __attribute__((address_space(3))) P*;
    const float* arow = W + (2 * i - 1 + r + 2 * R) * M::AP + CA + c0;
    const P lo = *(LP)(arow - 2), mid = *(LP)arow, hi = *(LP)(arow + 2);
    y[0] = lo[1];
    y[1] = mid[0];
    y[2] = mid[1];
    y[3] = hi[0];
  };
  auto qrow = [&](int r, const float(&yr)[4], const float(&yn)[4], float(&q0)[3], float(&q1)[3]) {
#pragma unroll
    for (int c = 0; c <= 2; ++c) {
      const float v0 = fma(p->g0a, yr[c], p->g0b * yn[c]);
      const float v1 = fma(p->g1a, yr[c], p->g1b * yr[c + 1]);
      float w = tv_weight<float>(fma(v0, v0, v1 * v1), p->lam, p->mu, p->inv_mu);
      if (EDGE) {
        const int gr = r0 + 2 * i - 1 + r, gc = tx0 + c0 - 1 + c;
        if (!(gr >= 0 && gr < n0 && gc >= 0 && gc < n1)) w = 0.0f;
      }
      q0[c] = v0 * w;
      q1[c] = v1 * w;
    }
  };
  float tv[2][2];
  const bool use_tv = p->tv && tv_on;
  if (use_tv) {
    float yr[4], yn[4];
    yrow(0, yr);
    yrow(1, yn);
    float qp0[3], qp1[3];
    qrow(0, yr, yn, qp0, qp1);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int c = 0; c < 4; ++c) yr[c] = yn[c];
      yrow(u + 2, yn);
      float qc0[3], qc1[3];
      qrow(u + 1, yr, yn, qc0, qc1);
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        const float t0 = fma(p->g0b, qp0[w + 1], p->g0a * qc0[w + 1]);
        const float t1 = fma(p->g1b, qc1[w], p->g1a * qc1[w + 1]);
        tv[u][w] = t0 + t1;
      }
#pragma unroll
      for (int c = 0; c <= 2; ++c) qp0[c] = qc0[c];
    }
  }
  float acc[2][2];  // acc[w][u]: column c0 + w, band row 2i + u
  sweep2<R, 2, M::PTP>(PT + (CA - 2 * R + c0) * M::PTP + 2 * i, p->g1, acc);
  const bool edge_cols = EDGE && (tx0 < R || tx0 + TX > n1 - R);
  if (edge_cols) ghost_cols_fix<R, 2>(tx0 + c0, n1, 2 * i, KT + M::GH_OFF - M::KT_OFF, KT + kKT, acc);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    float g0 = acc[0][u], g1 = acc[1][u];
    if (use_tv) {
      g0 = g0 + tv[u][0];
      g1 = g1 + tv[u][1];
    }
    *reinterpret_cast<float2*>(O + M::oidx(2 * i + u, c0)) = make_float2(g0, g1);
  }
}

// One workgroup's run of nb bands of one strip.  EDGE: some band of the run touches the image border
// (zero-page DMA granules, boundary corrections, masked TV weights and stores); the interior runs -- all
// but the first / last strips and runs of a large image -- take the branch-free instantiation.
template <int R, bool EDGE>
__device__ inline void march_run(const PgdParams<float>& p, float* smem, int kb0, int nb, int tx0, const float* xs,
                                 const float* xps, const float* bs, float* xns, int diag) {
  using M = March<R>;
  float* W = smem + M::W_OFF;
  float* S = smem + M::S_OFF;
  float* PT = smem + M::PT_OFF;
  float* O = smem + M::O_OFF;
  float* KT = smem + M::KT_OFF;
  const int tid = threadIdx.x;
  const int n0 = p.n0, n1 = p.n1;
  auto issue_band = [&](int r0) {  // the band's 16 new window rows: image rows r0 + 2R ..
    if (diag & 2) return;
    march_issue<R, EDGE>(S, xs, xps, r0 + 2 * R, tx0, n0, n1);
  };
  const float a = p.a;
  // prologue: DMA of band 0's new rows, then the first SH window rows (image rows r0 - 2R ..) as yk
  int r0 = kb0 * M::TB;
  issue_band(r0);
  {
    constexpr int NV = M::SH * M::SV;
#pragma unroll
    for (int k = 0; k < cdiv(NV, kThreads); ++k) {
      const int q = tid + k * kThreads;
      if (q < NV) {
        const int r = q / M::SV, g = q - r * M::SV;
        const int gr = r0 - 2 * R + r, gc = tx0 - M::CA + 4 * g;
        float xv[4] = {0.f, 0.f, 0.f, 0.f}, pv[4] = {0.f, 0.f, 0.f, 0.f}, out[4];
        if (!EDGE || (gr >= 0 && gr < n0 && gc >= 0 && gc < n1)) {
          ld_vec<float, 4>(xs + (unsigned)(gr * n1 + gc), xv);
          ld_vec<float, 4>(xps + (unsigned)(gr * n1 + gc), pv);
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          out[v] = fma(xv[v] - pv[v], a, xv[v]);
        }
        st_vec<float, 4>(W + (M::TB + r) * M::AP + 4 * g, out);  // where band 0's shift picks them up
      }
    }
  }
  int el = 0, eq = 0;  // row-major epilogue lane: band row el, 16-B column vector eq
  Stage<float, 6>::lane(tid, el, eq);
  const KP kp = (KP)__builtin_amdgcn_kernarg_segment_ptr();  // p is the first kernel argument
  unsigned long long* ts = reinterpret_cast<unsigned long long*>(smem + M::BYTES / 4);
  const bool tracing = (diag & 32) != 0;
  auto mark = [&](int k, int pt) {
    if (tracing && (tid & 63) == 0 && k < 16) ts[((tid >> 6) * 16 + k) * 8 + pt] = clock64();
  };
  for (int k = 0; k < nb; ++k, r0 += M::TB) {
    const bool has_next = k + 1 < nb;
    mark(k, 0);
    // shift sources (W rows TB .. TB + SH - 1; band 0: the prologue's rows) into registers before the barrier
    constexpr int NSH = M::SH * M::SV;
    constexpr int KSH = cdiv(NSH, kThreads);
    f32x4 shv[KSH];
#pragma unroll
    for (int q = 0; q < KSH; ++q) {
      const int t = tid + q * kThreads;
      shv[q] = *reinterpret_cast<const f32x4*>(W + (M::TB + (t < NSH ? t / M::SV : 0)) * M::AP + 4 * (t < NSH ? t % M::SV : 0));
    }
    if (k > 0) wait_vm<1>();  // this wave's DMA(k) landed; band k-1's x_new store may stay in flight
    else wait_vm<0>();
    lds_barrier();  // B1: every wave's DMA(k) landed; band k-1 is done with W / PT / O
    mark(k, 1);
    // H^T y of this band's epilogue pixels, into registers (counted by hand)
    f32x4 bq;
    {
      const int gr = r0 + el, gc = tx0 + 4 * eq;
      const float* ptr = (!EDGE || (gr < n0 && gc < n1)) ? bs + (unsigned)(gr * n1 + gc) : g_zero_page;
      asm_load_b4(bq, ptr);
    }
#pragma unroll
    for (int q = 0; q < KSH; ++q) {
      const int t = tid + q * kThreads;
      if (t < NSH) {
        const int r = t / M::SV, g = t - r * M::SV;
        *reinterpret_cast<f32x4*>(W + r * M::AP + 4 * g) = shv[q];
      }
    }
    {  // S -> yk rows SH .. SH + TB - 1 of W
#pragma unroll
      for (int q = 0; q < cdiv(M::SSLOTS, kThreads); ++q) {
        const int t = tid + q * kThreads;
        if (t < M::SSLOTS) {
          const int r = t / M::SV, g = t - r * M::SV;
          float xv[4], pv[4], out[4];
          ld_vec<float, 4>(S + 4 * t, xv);
          ld_vec<float, 4>(S + 4 * (M::SSLOTS + t), pv);
#pragma unroll
          for (int v = 0; v < 4; ++v) out[v] = fma(xv[v] - pv[v], a, xv[v]);
          st_vec<float, 4>(W + (M::SH + r) * M::AP + 4 * g, out);
        }
      }
    }
    lds_barrier();  // B2: W complete, S read by every wave
    mark(k, 2);
    if (has_next) issue_band(r0 + M::TB);
    if (!(diag & 5)) march_pass_a<R, EDGE>(kp, W, PT, KT, r0);
    mark(k, 3);
    lds_barrier();  // B3: PT complete
    if (EDGE && (tx0 < R || tx0 + TX > n1 - R)) {  // edge strips: the boundary-column ghost terms
      march_ghost_cols<R>(kp, PT, smem + M::GH_OFF, tx0, n1);
      lds_barrier();
    }
    mark(k, 4);
    if (!(diag & 9)) march_pass_b<R, EDGE>(kp, W, PT, KT, O, r0, tx0, (diag & 16) == 0);
    mark(k, 5);
    lds_barrier();  // B4: O complete
    if (has_next) wait_vm<M::NDW>();  // H^T y landed; DMA(k+1) may stay in flight
    else wait_vm<0>();
    mark(k, 6);
    asm volatile("" : "+v"(bq));
    {
      float g[4], y[4];
      ld_vec<float, 4>(O + M::oidx(el, 4 * eq), g);
      ld_vec<float, 4>(W + (el + 2 * R) * M::AP + M::CA + 4 * eq, y);
      const float bv[4] = {bq[0], bq[1], bq[2], bq[3]};
      const float tau = kp->tau, pw = kp->pw;
      const int prox = kp->prox;
      float xo[4];
#pragma unroll
      for (int w = 0; w < 4; ++w) {  // finish_run's arithmetic
        float gsum = g[w] - bv[w];
        float z = fma(gsum, -tau, y[w]);
        xo[w] = apply_prox<float>(prox, z, pw);
      }
      const int gr = r0 + el, gc = tx0 + 4 * eq;
      // exactly ONE store instruction per lane and band, whatever the lane's position (the top-of-band
      // wait counts it): out-of-image lanes write the sink page (n1 % 4 == 0: a vector is wholly in or out)
      float* dst = (!EDGE || (gr < n0 && gc < n1)) ? xns + (unsigned)(gr * n1 + gc) : g_sink_page;
      *reinterpret_cast<float4*>(dst) = make_float4(xo[0], xo[1], xo[2], xo[3]);
    }
    mark(k, 7);
  }
  if (tracing && (blockIdx.x == 0 || blockIdx.x == gridDim.x / 2)) {
    lds_barrier();
    const int base = blockIdx.x == 0 ? 0 : kTraceWords / 2;
    for (int q = tid; q < kTraceWords / 2; q += kThreads) g_march_trace[base + q] = ts[q];
  }
}

template <int R>
__global__ void __launch_bounds__(kThreads, 4) pgd_march_kernel(PgdParams<float> p, const float* __restrict__ x,
                                                              const float* __restrict__ xp,
                                                              const float* __restrict__ b, float* __restrict__ xn,
                                                              int sb, int nseg, int nstrips, unsigned nunits,
                                                              int diag) {
  using M = March<R>;
  extern __shared__ __attribute__((aligned(16))) float smem_m[];
  const int tid = threadIdx.x;
  const int n0 = p.n0, n1 = p.n1;
  const unsigned unit = xcd_tile(blockIdx.x, nunits);
  const unsigned per_img = (unsigned)nseg * (unsigned)nstrips;
  const unsigned s = unit / per_img;
  const unsigned rem = unit - s * per_img;
  const int seg = (int)(rem / (unsigned)nstrips);
  const int tx0 = (int)(rem - (unsigned)seg * (unsigned)nstrips) * TX;
  const int nbands = (n0 + M::TB - 1) / M::TB;
  const int kb0 = seg * sb;
  const int nb = (kb0 + sb <= nbands ? sb : nbands - kb0);
  const int64_t img = (int64_t)n0 * n1;
  const float* xs = x + (int64_t)s * img;
  const float* xps = xp + (int64_t)s * img;
  const float* bs = b + (int64_t)(s % (unsigned)p.y_images) * img;
  float* xns = xn + (int64_t)s * img;
  float* KT = smem_m + M::KT_OFF;
  if (tid < 2 * R + 1) {
    KT[tid] = p.k0[tid];
    KT[kKT + tid] = p.k1[tid];
  }
  const bool interior = tx0 - M::CA >= 0 && tx0 + TX + M::CA <= n1 && kb0 * M::TB - 2 * R >= 0 &&
                        (kb0 + nb) * M::TB + 2 * R <= n0;
  if (interior) march_run<R, false>(p, smem_m, kb0, nb, tx0, xs, xps, bs, xns, diag);
  else march_run<R, true>(p, smem_m, kb0, nb, tx0, xs, xps, bs, xns, diag);
}

struct MarchPlan {
  int sb, nseg, nstrips;
  unsigned nunits;
};

// bands per workgroup: enough units for ~4 workgroups per CU, whole strips at most
inline int march_plan(int64_t stack, int n0, int n1, MarchPlan& mp) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return PXA_ERR_UNSUPPORTED;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
  }
  const int64_t nbands = (n0 + 15) / 16;
  mp.nstrips = (n1 + TX - 1) / TX;
  const int64_t total = stack * nbands * mp.nstrips;
  int64_t sb = (total + 4 * (int64_t)cus - 1) / (4 * (int64_t)cus);
  if (tuning(PXA_TUNE_MARCH_BANDS) > 0) sb = tuning(PXA_TUNE_MARCH_BANDS);
  sb = sb < 1 ? 1 : (sb > nbands ? nbands : sb);
  mp.sb = (int)sb;
  mp.nseg = (int)((nbands + sb - 1) / sb);
  const int64_t nu = stack * mp.nseg * mp.nstrips;
  if (nu > 0x7fffffff) return PXA_ERR_UNSUPPORTED;
  mp.nunits = (unsigned)nu;
  return PXA_OK;
}

template <int R>
int launch_pgd_march(const PgdParams<float>& p, const void* x, const void* xp, const void* b, void* xn,
                     hipStream_t s) {
  using M = March<R>;
  auto kern = pgd_march_kernel<R>;
  static bool attr_set = false;
  if (!attr_set) {  // room for the timing trace (diag bit 5) beyond the kernel's own carve
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(M::BYTES + kTraceWords / 2 * 8));
    attr_set = true;
  }
  const int diag = tuning(PXA_TUNE_PGD_DIAG);
  const size_t smem = M::BYTES + ((diag & 32) ? kTraceWords / 2 * 8 : 0);
  MarchPlan mp;
  const int st = march_plan(p.stack, p.n0, p.n1, mp);
  if (st != PXA_OK) return st;
  hipLaunchKernelGGL(kern, dim3(mp.nunits), dim3(kThreads), smem, s, p, (const float*)x, (const float*)xp,
                     (const float*)b, (float*)xn, mp.sb, mp.nseg, mp.nstrips, mp.nunits, diag);
  return last_launch_status();
}


thread_local int g_last_pgd_kernel = 0;  // pxa_pgd_tv2d_last_kernel

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
  p.diag = tuning(PXA_TUNE_PGD_DIAG);
  if constexpr (sizeof(T) == 4) {
    // march kernel (PXA_TUNE_PGD_KERNEL = 5 forces it where it applies): fp32, R <= 6, 16-B rows,
    // 32-bit in-image offsets, no RelError partials
    const int knob = tuning(PXA_TUNE_PGD_KERNEL);
    if (p.vec_ok && n0 * n1 <= 0x7fffffff && R <= 6 && partials == nullptr && knob == 5) {
      int st;
      switch (R) {
        case 1: st = launch_pgd_march<1>(p, x, x_prev, hty, x_new, s); break;
        case 2: st = launch_pgd_march<2>(p, x, x_prev, hty, x_new, s); break;
        case 3: st = launch_pgd_march<3>(p, x, x_prev, hty, x_new, s); break;
        case 4: st = launch_pgd_march<4>(p, x, x_prev, hty, x_new, s); break;
        case 5: st = launch_pgd_march<5>(p, x, x_prev, hty, x_new, s); break;
        default: st = launch_pgd_march<6>(p, x, x_prev, hty, x_new, s); break;
      }
      if (st == PXA_OK) g_last_pgd_kernel = 2;
      return st;
    }
  }
  int st;
  switch (R) {
    case 1: st = launch_pgd<T, 1>(p, x, x_prev, hty, x_new, partials, s); break;
    case 2: st = launch_pgd<T, 2>(p, x, x_prev, hty, x_new, partials, s); break;
    case 3: st = launch_pgd<T, 3>(p, x, x_prev, hty, x_new, partials, s); break;
    case 4: st = launch_pgd<T, 4>(p, x, x_prev, hty, x_new, partials, s); break;
    case 5: st = launch_pgd<T, 5>(p, x, x_prev, hty, x_new, partials, s); break;
    case 6: st = launch_pgd<T, 6>(p, x, x_prev, hty, x_new, partials, s); break;
    case 7: st = launch_pgd<T, 7>(p, x, x_prev, hty, x_new, partials, s); break;
    default: st = launch_pgd<T, 8>(p, x, x_prev, hty, x_new, partials, s); break;
  }
  if (st == PXA_OK) g_last_pgd_kernel = 1;
  return st;
}

}  // namespace
}  // namespace pxa

using namespace pxa;

extern "C" {

int pxa_pgd_tv2d_last_kernel(void) { return g_last_pgd_kernel; }

int pxa_pgd_march_trace(uint64_t* host_out, int n) {
  if (!host_out || n < 0 || n > kTraceWords) return PXA_ERR_ARG;
  if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_march_trace), (size_t)n * 8, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return PXA_ERR_UNSUPPORTED;
  return PXA_OK;
}

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
