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

// Wave priority (s_setprio) of the window-load phase: its loads issue ahead of the passes of the other
// workgroups resident on the SIMD, so that the next round's windows are in flight sooner.  Interleaved A/B
// (profiles/r05zb_pgd_prio_ab.txt): 2048^2 24.4 -> 23.4 us on one box, no change on another (r05zc); C5 and
// 4096^2 unchanged within noise; priority 2 or 3, or also raising the epilogue, gave the same.  Scheduling
// only: the same bits.
#ifndef PXA_PGD_PRIO
#define PXA_PGD_PRIO 1
#endif
#ifndef PXA_PGD_PRIO_EPI
#define PXA_PGD_PRIO_EPI 0  // (A/B builds: the epilogue's H^T y loads too)
#endif
#ifndef PXA_PGD_PRIO_FIN
#define PXA_PGD_PRIO_FIN 0  // (A/B builds: the finishing row-major epilogue)
#endif

// Measurement probes (s_memtime phase trace, skip probes, staggered starts: PXA_TUNE_PGD_DIAG /
// PXA_TUNE_PGD_STAGGER) exist only in the probe build (`make -C pyxu_amd/csrc probe`, scripts/ that time
// kernel phases); the production library compiles them out, so its kernel carries no probe branch.
#ifndef PXA_PROBES
#define PXA_PROBES 0
#endif

namespace pxa {
namespace {

using namespace tile2d;
constexpr bool kProbes = PXA_PROBES != 0;


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
  int diag;     // PXA_TUNE_PGD_DIAG (bit 5: s_memtime phase trace of a few workgroups)
  int stagger;  // PXA_TUNE_PGD_STAGGER (A/B probe: delayed start of some first-round workgroups)
  unsigned round1;  // workgroups resident at once (4 per CU)
  const T* xref;    // RelError partials relative to this iterate (nullptr: relative to x)
  // last-workgroup fold of the RelError partials (pxa_pgd_tv2d_plan_step with rel_values): the workgroup
  // that finishes last folds them as pxa_tile_partials_fold does (same bits) into fold_vals (host-mapped,
  // (2, fold_rows)) and sets fold_flags[q] = fold_seq; `counter` (device, 0 between launches) counts the
  // finished workgroups.  fold_vals == nullptr: no fold.
  double* fold_vals;
  unsigned* fold_flags;
  unsigned* counter;
  unsigned fold_seq;
  int64_t fold_rows, fold_per_row;
  // strip kernel (pgd_strip_kernel): tiles per strip, strip groups per tile column of an image, strips in all
  unsigned slen, sgroups, nstrips;
  // pipelined kernel (pgd_pipe_kernel): resident tile workgroups (0: not that kernel)
  unsigned pipe_wgs;
  // window partials (pxa_pgd_tv2d_plan_step_wfold): the per-(tile, wave) partials are (sum (x - x_prev)^2, sum x_prev^2)
  // over the tile, from the window loads -- the RelError statistics of the PREVIOUS step's check -- instead of the
  // epilogue's (x_new - x_ref) statistics: no extra load of x
  int win_part;
  // publication of the PREVIOUS launch's partials (pxa_pgd_tv2d_plan_step_wpub): one extra workgroup (block ntiles)
  // folds pub_src as pxa_tile_partials_fold does (same bits) into pub_vals and sets pub_flags[q] = pub_seq, beside
  // the tile workgroups -- no fold launch, no cross-workgroup hand-off (pub_src is complete at launch)
  const double* pub_src;
  double* pub_vals;
  unsigned* pub_flags;
  unsigned pub_seq;
};

// Round 3 also measured a variant that carried yk as solver state (the epilogue writing the next
// iteration's yk, the window reading one array instead of two): equal at 2048^2 (25.4 vs 24.9 us) and
// slower at 4096^2 (79.6 vs 66.2 us), where the fifth compulsory stream costs more than the halved window
// saves; it was removed.

// Timing trace (PXA_TUNE_PGD_DIAG bit 5, read by pxa_pgd_tile_trace): s_memtime stamps of waves 0-3 of
// workgroups 0, 1, grid/2 and grid-1, 8 points of their tile.  Staged in LDS beyond the kernel's own
// carve, dumped at exit.
constexpr int kTraceWords = 4 * 4 * 8;
__device__ unsigned long long g_tile_trace[kTraceWords];

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
  return lam * __builtin_fminf(r, inv_mu);      // one v_min_f32 (r is never NaN: n2 >= 0)
}

// ---- phase 0 of the tile kernel: yk = (x - x_prev) * a + x on the A window, zero outside the image.
// All K0 vector pairs of a thread are loaded before the first LDS store, so their latencies overlap.
// `lt`: the thread's index among the kThreads threads that share the window.
template <typename T, int R>
struct Window {
  using L = Layout<T, R>;
  static constexpr int K0 = cdiv(L::N0, kThreads);
  // the tile's own vectors come first (thread-uniform: items k < KI of every thread), then the halo
  static constexpr int NI = TY * (TX / L::V);
  static constexpr int KI = NI / kThreads;
  static_assert(NI % kThreads == 0, "every thread loads KI of the tile's own vectors");
  T xv[K0][L::V], pv[K0][L::V];
};

// Window vector `it` (0 .. N0) -> window row r, vector column g.  Items 0 .. NI - 1 are the tile's own TY x TX pixels
// (row-major), the rest the halo: the top 2R rows, then the CA / V vectors left and right of each tile row, then the
// bottom 2R rows.  So the RelError window partials (the tile's pixels only) are items k < KI of every thread: no
// divergent double-precision code (the row-major order spread them over all K0 items, exec-masked).  Any bijection
// gives the same A (each vector's yk is computed alone): the order only moves work between threads.
#ifndef PXA_PGD_WIN_ROWMAJOR
#define PXA_PGD_WIN_ROWMAJOR 0  // (A/B builds: the row-major window order of rounds 1-5)
#endif
template <typename T, int R>
__device__ inline void win_rg(int it, int& r, int& g) {
  using L = Layout<T, R>;
  if (PXA_PGD_WIN_ROWMAJOR) {
    r = it / L::NGA;
    g = it - r * L::NGA;
    return;
  }
  constexpr int TV = TX / L::V, CV = L::CA / L::V, NI = Window<T, R>::NI;
  constexpr int TOP = 2 * R * L::NGA, MID = TY * 2 * CV;
  if (it < NI) {
    r = 2 * R + it / TV;
    g = CV + it % TV;
    return;
  }
  const int h = it - NI;
  if (h < TOP) {
    r = h / L::NGA;
    g = h - r * L::NGA;
  } else if (h < TOP + MID) {
    const int m = h - TOP, q = m % (2 * CV);
    r = 2 * R + m / (2 * CV);
    g = q < CV ? q : q + TV;
  } else {
    const int b = h - TOP - MID, rb = b / L::NGA;
    r = 2 * R + TY + rb;
    g = b - rb * L::NGA;
  }
}

template <typename T, int R, bool EDGE>
__device__ inline void win_issue(const PgdParams<T>& p, int ty0, int tx0, const T* __restrict__ xs,
                                 const T* __restrict__ xps, Window<T, R>& w, int lt) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
  constexpr int CA = L::CA;
  const int n0 = p.n0, n1 = p.n1;
#pragma unroll
  for (int k = 0; k < Window<T, R>::K0; ++k) {
    const int it = lt + k * kThreads;
    if (it < L::N0) {
      int r, g;
      win_rg<T, R>(it, r, g);
      const int gr = ty0 - 2 * R + r, gc = tx0 - CA + V * g;
      if (!EDGE) {
        const unsigned off = (unsigned)(gr * n1 + gc);
        ld_vec<T, V>(xs + off, w.xv[k]);
        if (kProbes && (p.diag & 256)) {  // timing probe only (WRONG results): one window array instead of two
#pragma unroll
          for (int v = 0; v < V; ++v) w.pv[k][v] = w.xv[k][v];
        } else {
          ld_vec<T, V>(xps + off, w.pv[k]);
        }
      } else if (gr >= 0 && gr < n0 && p.vec_ok && gc >= 0 && gc + V <= n1) {
        ld_vec<T, V>(xs + (int64_t)gr * n1 + gc, w.xv[k]);
        ld_vec<T, V>(xps + (int64_t)gr * n1 + gc, w.pv[k]);
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const bool in = gr >= 0 && gr < n0 && gc + v >= 0 && gc + v < n1;
          w.xv[k][v] = in ? xs[(int64_t)gr * n1 + gc + v] : T(0);
          w.pv[k][v] = in ? xps[(int64_t)gr * n1 + gc + v] : T(0);
        }
      }
    }
  }
}

template <typename T, int R>
__device__ inline void win_store(const PgdParams<T>& p, T* A, const Window<T, R>& w, int lt) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
#pragma unroll
  for (int k = 0; k < Window<T, R>::K0; ++k) {
    const int it = lt + k * kThreads;
    if (it < L::N0) {
      int r, g;
      win_rg<T, R>(it, r, g);
      T out[V];
#pragma unroll
      for (int v = 0; v < V; ++v) out[v] = fma(w.xv[k][v] - w.pv[k][v], p.a, w.xv[k][v]);  // one rounding site
      st_vec<T, V>(A + r * L::AP + V * g, out);
    }
  }
}

template <typename T, int R, bool EDGE>
__device__ inline void load_window(const PgdParams<T>& p, T* A, int ty0, int tx0, const T* __restrict__ xs,
                                   const T* __restrict__ xps) {
  Window<T, R> w;
  win_issue<T, R, EDGE>(p, ty0, tx0, xs, xps, w, threadIdx.x);
  win_store<T, R>(p, A, w, threadIdx.x);
}

// ---- pass A: PT[col][row] = (G0 yk)[row][col] for the TY tile rows and all A columns
template <typename T, int R, bool EDGE, int D = 0>
__device__ inline void pass_a(const PgdParams<T>& p, const T* A, T* PT, const T* KT, int ty0, int tid = threadIdx.x) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
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
      sweep<T, R, V, L::AP, D>(A + (V * a) * L::AP + V * b, p.g0, acc);
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

// ---- TV dual once per pixel (fp32 lane map of pass B; PXA_PGD_TVX=0 builds the 5 x 3 window path for A/B).  Pass B's item (4 rows x 2
// columns) needs q at its own 8 pixels, q0 one row above and q1 one column to the left; the default path
// evaluates q on the 5 x 3 window (15 per item, 1.9 x per pixel).  Here an item evaluates its own 8, writes
// its last row's q0 and last column's q1 to an exchange area in A's rows that pass B no longer reads, lanes
// 0..47 of the wavefront evaluate the wavefront's halo (16 q0 of the tile row above, 32 q1 of the column to the
// left of the wavefront's 16 columns), and every item reads its neighbours' values back.  Same q expressions,
// same bits.  Within one wavefront (items (a, cb) of a wavefront: all 8 row groups x 8 column items) LDS
// accesses execute in order, so no barrier is needed.  Interleaved A/B (r05zj, profiles/r05zj_pgd_tvx_ab.txt):
// bit-identical at 2048^2 and 1000 x 1500; kernel 23.5 -> 23.3 us at 2048^2, C5 0.657 -> 0.651 ms, 4096^2 76.6 ->
// 72.9 us: the VALU saved is partly spent on the exchange's LDS traffic.
#ifndef PXA_PGD_TVX
#define PXA_PGD_TVX 1
#endif
constexpr int kTvxFloats = 9 * 16 + 9 * 32;  // per wavefront: q0 [row group + 1][16 cols], q1 [col item + 1][32 rows]

template <typename T, int R, bool EDGE>
__device__ inline void tv_exchange(const PgdParams<T>& p, T* A, int ty0, int tx0, int tid, int a, int cb,
                                   T (&yc)[kVecN<T>][2], T (&tv)[kVecN<T>][2], T* xarea23) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
  constexpr int CA = L::CA;
  const int n0 = p.n0, n1 = p.n1;
  const int lane = tid & 63, wv = tid >> 6, cbl = cb & 7;
  const int c0 = 2 * cb;
  // own rows (window rows 1..V) and the row below, columns c0 .. c0 + 2
  T y[V + 1][3];
#pragma unroll
  for (int r = 0; r <= V; ++r) {
    const T* arow = A + (V * a + r + 2 * R) * L::AP + CA + c0;
    T mid[2], hi[2];
    ld_pair<T>(arow, mid);
    ld_pair<T>(arow + 2, hi);
    y[r][0] = mid[0];
    y[r][1] = mid[1];
    y[r][2] = hi[0];
  }
#pragma unroll
  for (int u = 0; u < V; ++u)
#pragma unroll
    for (int w = 0; w < 2; ++w) yc[u][w] = y[u][w];
  if (!p.tv) return;
  auto qat = [&](T yc_, T ydn, T yrt, int gr, int gc, T& q0, T& q1) {
    const T v0 = fma(p.g0a, yc_, p.g0b * ydn);
    const T v1 = fma(p.g1a, yc_, p.g1b * yrt);
    T w = tv_weight<T>(fma(v0, v0, v1 * v1), p.lam, p.mu, p.inv_mu);
    if (EDGE && !(gr >= 0 && gr < n0 && gc >= 0 && gc < n1)) w = T(0);
    q0 = v0 * w;
    q1 = v1 * w;
  };
  T q0[V][2], q1[V][2];
#pragma unroll
  for (int u = 0; u < V; ++u)
#pragma unroll
    for (int w = 0; w < 2; ++w)
      qat(y[u][w], y[u + 1][w], y[u][w + 1], ty0 + V * a + u, tx0 + c0 + w, q0[u][w], q1[u][w]);
  // exchange area of this wavefront: waves 0, 1 in A's top dead rows, 2, 3 in the bottom ones -- or, in the strip
  // kernel (whose bottom window rows are the next tile's top rows), in `xarea23` beside the tile's LDS carve
  T* E = (wv < 2 ? A : xarea23 != nullptr ? xarea23 : A + (TY + 2 * R + 1) * L::AP) + (wv & 1) * kTvxFloats;
  T* E0 = E;            // [a + 1][col within the wavefront's 16]
  T* E1 = E + 9 * 16;   // [col item + 1][row]
  // halo of the wavefront: lanes 0..15 the q0 of tile row -1 (its 16 columns), lanes 16..47 the q1 of the column
  // left of its first column (tile rows 0..31)
  if (lane < 48) {
    T hq0, hq1;
    if (lane < 16) {
      const int tc = 16 * wv + lane;
      const T* r0 = A + (2 * R - 1) * L::AP + CA + tc;
      qat(r0[0], r0[L::AP], r0[1], ty0 - 1, tx0 + tc, hq0, hq1);
      E0[lane] = hq0;
    } else {
      const int j = lane - 16, tc = 16 * wv - 1;
      const T* r0 = A + (j + 2 * R) * L::AP + CA + tc;
      qat(r0[0], r0[L::AP], r0[1], ty0 + j, tx0 + tc, hq0, hq1);
      E1[j] = hq1;
    }
  }
  {
    const T b[2] = {q0[V - 1][0], q0[V - 1][1]};
    st_vec<T, 2>(E0 + (a + 1) * 16 + 2 * cbl, b);
    const T c[4] = {q1[0][1], q1[1][1], q1[2][1], q1[3][1]};
    st_vec<T, 4>(E1 + (cbl + 1) * 32 + 4 * a, c);
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  T up[2], left[4];
  ld_vec<T, 2>(E0 + a * 16 + 2 * cbl, up);
  ld_vec<T, 4>(E1 + cbl * 32 + 4 * a, left);
#pragma unroll
  for (int u = 0; u < V; ++u)
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      const T qa = u == 0 ? up[w] : q0[u - 1][w];
      const T ql = w == 0 ? left[u] : q1[u][0];
      const T t0 = fma(p.g0b, qa, p.g0a * q0[u][w]);
      const T t1 = fma(p.g1b, ql, p.g1a * q1[u][w]);
      tv[u][w] = t0 + t1;
    }
}

// ---- pass B: G1 along rows + Grad^T q, handed per output row-run to
// `emit(k, u, gr, gc, g, yc)`: g = (G yk + Grad^T q) at row gr, columns gc .. gc + CW - 1 of item k,
// yc = yk there.  The emitter finishes the pixels in place (finish_run) or stages g for the
// coalesced epilogue (epilogue_staged).
template <typename T, int R, bool EDGE, typename Emit, int D = 0>
__device__ inline void pass_b(const PgdParams<T>& p, const T* A, const T* PT, const T* KT, const T* GH, int ty0, int tx0,
                              Emit&& emit, int tid = threadIdx.x, T* xarea23 = nullptr) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
  constexpr int CA = L::CA;
  constexpr int CW = L::CW;
  const int n0 = p.n0, n1 = p.n1;
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
      constexpr bool kX = PXA_PGD_TVX && sizeof(T) == 4 && L::NA == 8 && CW == 2 && KB == 1 &&
                          (2 * R - 1) * L::AP >= kTvxFloats * 2;
      if constexpr (kX) {
        tv_exchange<T, R, EDGE>(p, const_cast<T*>(A), ty0, tx0, tid, a, cb, yc, tv, xarea23);
      } else {
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
      sweep<T, R, CW, L::PTP, D>(PT + (CA - 2 * R + c0) * L::PTP + V * a, p.g1, acc);
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
// each 16-B vector of a row is one lane (16 lanes per fp32 row), so the H^T y / x loads and the x_new
// stores are full 128-B lines instead of the pass-B item order's 64-B row pieces (measured on MI355X: a
// 2048^2 fp32 store in the item order 7.2 us, row-major 5.2 us).  yk comes from A.
// StagedB: H^T y (and x, when the RelError partials need it) of this thread's epilogue vectors, zero
// outside the image; H^T y is issued before the O staging so that its latency overlaps it.
template <typename T, int R>
struct StagedB {
  static constexpr int NS = TY / Stage<T, R>::RPS;
  T v[NS][kVecN<T>];
  T x[NS][kVecN<T>];
};

// a whole 16-B vector of row gr at column gc lies inside the image and can be moved as one access
template <typename T>
__device__ inline bool vec_inside(const PgdParams<T>& p, int gr, int gc) {
  return p.vec_ok && gr < p.n0 && gc + kVecN<T> <= p.n1;
}

template <typename T, int R, bool EDGE>
__device__ inline void load_staged(const PgdParams<T>& p, int ty0, int tx0, const T* __restrict__ src, T (&v)[StagedB<T, R>::NS][kVecN<T>],
                                   int lt = threadIdx.x) {
  using S = Stage<T, R>;
  constexpr int V = kVecN<T>;
  const int n0 = p.n0, n1 = p.n1;
  int r0, cq;
  S::lane(lt, r0, cq);
#pragma unroll
  for (int s = 0; s < StagedB<T, R>::NS; ++s) {  // all loads first: one round trip
    const int gr = ty0 + r0 + s * S::RPS, gc = tx0 + V * cq;
    if (!EDGE) {
      ld_vec<T, V>(src + (unsigned)(gr * n1 + gc), v[s]);
    } else if (vec_inside(p, gr, gc)) {  // edge tile, but this vector is inside: one 16-B load
      ld_vec<T, V>(src + (int64_t)gr * n1 + gc, v[s]);
    } else {
#pragma unroll
      for (int w = 0; w < V; ++w) v[s][w] = (gr < n0 && gc + w < n1) ? src[(int64_t)gr * n1 + gc + w] : T(0);
    }
  }
}

// z = ((G yk + Grad^T q) - H^T y) * (-tau) + yk; x_new = prox(z); RelError partials sum (x_new - x)^2,
// sum x^2 in double.  One 16-B vector of one tile row.
template <typename T, bool EDGE>
__device__ inline void finish_vec(const PgdParams<T>& p, int gr, int gc, const T (&g)[kVecN<T>], const T (&bv)[kVecN<T>],
                                  const T (&yc)[kVecN<T>], const T (&xv)[kVecN<T>], T* __restrict__ xns,
                                  bool want_part, double& part_d, double& part_x) {
  constexpr int V = kVecN<T>;
  const int n0 = p.n0, n1 = p.n1;
  T xo[V];
#pragma unroll
  for (int w = 0; w < V; ++w) {
    const T gsum = g[w] - bv[w];  // (G yk + Grad^T q) - H^T y
    const T z = fma(gsum, -p.tau, yc[w]);
    xo[w] = apply_prox<T>(p.prox, z, p.pw);
  }
  const bool whole = !EDGE || vec_inside(p, gr, gc);
  if (whole) {
    st_vec<T, V>(xns + (EDGE ? (int64_t)gr * n1 + gc : (int64_t)(unsigned)(gr * n1 + gc)), xo);
    if (want_part) {
#pragma unroll
      for (int w = 0; w < V; ++w) {
        const double dd = (double)xo[w] - (double)xv[w];
        part_d = fma(dd, dd, part_d);  // explicit: the vector and scalar paths must contract alike
        part_x = fma((double)xv[w], (double)xv[w], part_x);
      }
    }
  } else if (gr < n0) {
#pragma unroll
    for (int w = 0; w < V; ++w) {
      if (gc + w < n1) {
        xns[(int64_t)gr * n1 + gc + w] = xo[w];
        if (want_part) {
          const double dd = (double)xo[w] - (double)xv[w];
          part_d = fma(dd, dd, part_d);
          part_x = fma((double)xv[w], (double)xv[w], part_x);
        }
      }
    }
  }
}

// RelError partials per wavefront: lane 0 of the wave writes its (sum (x_new - r)^2, sum r^2), r = x_ref or x, to
// partials[2 slot .. 2 slot + 1], slot = tile * kPartWaves + wave (fixed-order shuffle fold, no barrier).
constexpr int kPartWaves = kThreads / 64;

__device__ inline void wave_partials(double part_d, double part_x, double* partials, unsigned slot) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    part_d += __shfl_down(part_d, off, 64);
    part_x += __shfl_down(part_x, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    // relaxed device-scope atomic stores: written through to the memory side (past this XCD's L2), so that the
    // last-workgroup fold (tail_fold) on any XCD can read them without a release fence -- a device-scope fence
    // per workgroup writes back the whole L2 (r05f: the kernel took 242 us instead of 25 with one)
    __hip_atomic_store(partials + 2 * slot, part_d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(partials + 2 * slot + 1, part_x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Prefetch point of the strip kernel's next-window rows inside a tile (PXA_PGD_STRIP_ISSUE): 0 right after pass A
// (the loads overlap pass B and the epilogue, and occupy registers through pass B), 1 after the epilogue's own
// loads (they overlap the O staging and the finishing stores only).
#ifndef PXA_PGD_STRIP_ISSUE
#define PXA_PGD_STRIP_ISSUE 1
#endif
// Rows in flight per G sweep (tile2d.hpp sweep's D): 0 = compiler-scheduled (tile kernel default); the strip kernel
// limits it so that its prefetched rows fit beside the passes in 128 VGPRs
#ifndef PXA_PGD_SWEEP_DEPTH
#define PXA_PGD_SWEEP_DEPTH 0
#endif
#ifndef PXA_PGD_STRIP_DEPTH
#define PXA_PGD_STRIP_DEPTH 6
#endif

struct NoHook {
  __device__ void operator()() const {}
};

// Workgroup barrier of a tile body.  RB: the raw form (LDS operations complete, then s_barrier) for the pipelined
// kernel, whose next window is in flight by LDS-DMA during the body -- __syncthreads()'s fence would wait for it
// (an LDS-DMA is a pending LDS write on the VM counter) at every barrier.  The body's own global loads land in
// registers, which the compiler waits for at their use, so the raw form orders everything the body shares.
template <bool RB>
__device__ inline void body_sync() {
  if constexpr (RB) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  } else {
    __syncthreads();
  }
}

// The phases of one output tile once its window is in A (behind a barrier): pass A, [ghost columns], pass B
// (parked in registers), the H^T y / x loads, O staging, row-major epilogue, [RelError partials].  `mid` runs at the
// strip kernel's prefetch point; `xarea23`: see tv_exchange (nullptr in the tile kernel).
template <typename T, int R, bool EDGE, int D, bool RB, typename Mid>
__device__ inline void pgd_tile_body(const PgdParams<T>& p, unsigned char* smem, unsigned tile, int ty0, int tx0,
                                     const T* __restrict__ bs, T* __restrict__ xns, double* __restrict__ partials,
                                     const T* __restrict__ xrs, T* xarea23, Mid&& mid, const int tid) {
  using L = Layout<T, R>;
  using S = Stage<T, R>;
  constexpr int CW = L::CW;
  constexpr int V = L::V;
  constexpr int KB = cdiv(L::NPB, kThreads);
  T* A = reinterpret_cast<T*>(smem);
  T* PT = A + L::AR * L::AP;
  T* KT = PT + L::AC * L::PTP;  // H taps for runtime-indexed reads (boundary corrections)
  T* GH = reinterpret_cast<T*>(smem + kGhOff<T, R>);  // boundary-column ghost terms (edge-column tiles)
  const int n1 = p.n1;
  const bool edge_cols = EDGE && (tx0 < R || tx0 + TX > n1 - R);
  double part_d = 0.0, part_x = 0.0;
  const bool want_part = partials != nullptr;
  const bool tracing = kProbes && (p.diag & 32) != 0 && xarea23 == nullptr;
  unsigned long long* ts = reinterpret_cast<unsigned long long*>(smem + kGhOff<T, R> + kGhBytes<T, R>);
  auto tmark = [&](int pt) {
    if (tracing && (tid & 63) == 0) ts[(tid >> 6) * 8 + pt] = clock64();
  };
  tmark(2);
  const bool skip_passes = kProbes && (p.diag & 64) != 0;  // timing probe only (WRONG results)
  if (!skip_passes) pass_a<T, R, EDGE, D>(p, A, PT, KT, ty0, tid);
  tmark(3);
  body_sync<RB>();
  if (PXA_PGD_STRIP_ISSUE == 0) mid();
  if (edge_cols) {
    ghost_cols_coop<T, R>(p.k1, PT, GH, tx0, n1, tid);
    body_sync<RB>();
  }
  tmark(4);
  T st[KB][V][CW];
  if (skip_passes) {
#pragma unroll
    for (int k = 0; k < KB; ++k)
#pragma unroll
      for (int u = 0; u < V; ++u)
#pragma unroll
        for (int w = 0; w < CW; ++w) st[k][u][w] = A[tid + u * 64 + w];
  } else
  {
    auto park = [&](int k, int u, int, int, const T(&g)[CW], const T(&)[CW]) {
#pragma unroll
      for (int w = 0; w < CW; ++w) st[k][u][w] = g[w];
    };
    pass_b<T, R, EDGE, decltype(park)&, D>(p, A, PT, KT, GH, ty0, tx0, park, tid, xarea23);
  }
  StagedB<T, R> hb;
  if (kProbes && (p.diag & 512)) {  // timing probe only (WRONG results): no H^T y loads
#pragma unroll
    for (int s = 0; s < StagedB<T, R>::NS; ++s)
#pragma unroll
      for (int w = 0; w < kVecN<T>; ++w) hb.v[s][w] = T(0);
  } else {
#if PXA_PGD_PRIO_EPI
    __builtin_amdgcn_s_setprio(PXA_PGD_PRIO_EPI);
#endif
    load_staged<T, R, EDGE>(p, ty0, tx0, bs, hb.v, tid);  // in flight during the O staging
#if PXA_PGD_PRIO_EPI
    __builtin_amdgcn_s_setprio(0);
#endif
  }
  tmark(5);
  body_sync<RB>();  // every G1 sweep is done with PT: O may overwrite it
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
  // x (RelError partials only) is loaded once pass B's parked results are out of the registers
  if (want_part) load_staged<T, R, EDGE>(p, ty0, tx0, xrs, hb.x, tid);
  if (PXA_PGD_STRIP_ISSUE != 0) mid();
  body_sync<RB>();
  tmark(6);
#if PXA_PGD_PRIO_FIN
  __builtin_amdgcn_s_setprio(PXA_PGD_PRIO_FIN);  // A/B builds: the finishing stores ahead of other passes
#endif
  {
    int r0, cq;
    S::lane(tid, r0, cq);
#pragma unroll
    for (int s = 0; s < StagedB<T, R>::NS; ++s) {
      const int r = r0 + s * S::RPS;
      T g[V], y[V];
      ld_vec<T, V>(O + S::idx(r, V * cq), g);
      ld_vec<T, V>(A + (r + 2 * R) * L::AP + L::CA + V * cq, y);
      if (kProbes && (p.diag & 1024)) {  // timing probe only (WRONG results): no x_new stores
        if (g[0] + y[0] + hb.v[s][0] == T(-12345)) xns[0] = T(0);  // keeps the loads and the O / A reads
        continue;
      }
      finish_vec<T, EDGE>(p, ty0 + r, tx0 + V * cq, g, hb.v[s], y, hb.x[s], xns, want_part, part_d, part_x);
    }
  }
  tmark(7);
  if (want_part) wave_partials(part_d, part_x, partials, tile * kPartWaves + (tid >> 6));
  const unsigned nb = gridDim.x, bid = blockIdx.x;
  if (tracing && (bid == 0 || bid == 1 || bid == nb / 2 || bid == nb - 1)) {
    __syncthreads();
    const int slot = bid == 0 ? 0 : bid == 1 ? 1 : bid == nb / 2 ? 2 : 3;
    if (tid < 32) g_tile_trace[slot * 32 + tid] = ts[tid];
  }
}


// The previous check's RelError statistics over this tile's pixels, from its window (win_part): sum (x - x_prev)^2,
// sum x_prev^2 per wave (outside the image both are 0: no contribution).
template <typename T, int R>
__device__ inline void win_partials(const Window<T, R>& w, double* __restrict__ partials, unsigned tile, const int tid) {
  using L = Layout<T, R>;
  double part_d = 0.0, part_x = 0.0;
#pragma unroll
  for (int k = 0; k < (PXA_PGD_WIN_ROWMAJOR ? Window<T, R>::K0 : Window<T, R>::KI); ++k) {  // (items k < KI: the tile's own vectors, win_rg)
    int r = 2 * R, g = L::CA / L::V;
    if (PXA_PGD_WIN_ROWMAJOR) {
      const int it = tid + k * kThreads;
      if (it >= L::N0) continue;
      win_rg<T, R>(it, r, g);
    }
    if (r >= 2 * R && r < 2 * R + TY && L::V * g >= L::CA && L::V * g < L::CA + TX) {
#pragma unroll
      for (int v = 0; v < L::V; ++v) {
        const double dd = (double)w.xv[k][v] - (double)w.pv[k][v];
        part_d = fma(dd, dd, part_d);
        part_x = fma((double)w.pv[k][v], (double)w.pv[k][v], part_x);
      }
    }
  }
  // (DPP wave sums: the __shfl_down ladder of wave_partials is a chain of twelve LDS round trips, on the path to the
  // window's barrier here; the window statistics only have to agree with the epilogue ones to rounding)
  part_d = wave_sum_f64(part_d);
  part_x = wave_sum_f64(part_x);
  if ((tid & 63) == 0) {
    const unsigned slot = tile * kPartWaves + (tid >> 6);
    __hip_atomic_store(partials + 2 * slot, part_d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(partials + 2 * slot + 1, part_x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// One output tile of the tile kernel: phase 0 (window) into A, then the body.
template <typename T, int R, bool EDGE>
__device__ inline void pgd_tile(const PgdParams<T>& p, unsigned char* smem, unsigned tile, int ty0, int tx0,
                                const T* __restrict__ xs, const T* __restrict__ xps, const T* __restrict__ bs,
                                T* __restrict__ xns, double* __restrict__ partials, const T* __restrict__ xrs) {
  using L = Layout<T, R>;
  T* A = reinterpret_cast<T*>(smem);
  T* KT = A + L::AR * L::AP + L::AC * L::PTP;
  const int tid = threadIdx.x;
  if (EDGE && tid < 2 * R + 1) {
    KT[tid] = p.k0[tid];
    KT[kKT + tid] = p.k1[tid];
  }
  const bool tracing = kProbes && (p.diag & 32) != 0;
  unsigned long long* ts = reinterpret_cast<unsigned long long*>(smem + kGhOff<T, R> + kGhBytes<T, R>);
  auto tmark = [&](int pt) {
    if (tracing && (tid & 63) == 0) ts[(tid >> 6) * 8 + pt] = clock64();
  };
  tmark(0);
#if PXA_PGD_PRIO
  __builtin_amdgcn_s_setprio(PXA_PGD_PRIO);  // the window loads issue ahead of other workgroups' passes
#endif
  if (kProbes && (p.diag & 128)) {  // timing probe only (WRONG results): no window loads, yk = 0
    for (int i = tid; i < L::AR * L::AP; i += kThreads) A[i] = T(0);
  } else {
    Window<T, R> w;
    win_issue<T, R, EDGE>(p, ty0, tx0, xs, xps, w, tid);
    win_store<T, R>(p, A, w, tid);
    if (p.win_part && partials != nullptr) win_partials<T, R>(w, partials, tile, tid);
  }
#if PXA_PGD_PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
  tmark(1);
  __syncthreads();
  pgd_tile_body<T, R, EDGE, PXA_PGD_SWEEP_DEPTH, false>(p, smem, tile, ty0, tx0, bs, xns, p.win_part ? nullptr : partials, xrs,
                                                 nullptr, NoHook{}, tid);
}

// (Opt-in: PXA_RELERR_SINK=1; gfx950-specific.)  The hand-off below uses no release / acquire: it is the first row
// of the measured write-through hand-off table of MI355X_MICROARCH.md ("Workgroup dispatch, XCD placement &
// inter-workgroup visibility": one lane per storing workgroup signals with an agent-scope atomic add behind every
// storing wave's s_waitcnt vmcnt(0) and a workgroup barrier; all payload stores and loads are sc1, i.e. relaxed
// agent-scope atomics; the workgroup whose add returned last reads).  That form is measured on gfx950 / ROCm 7.2,
// not an architectural guarantee of the HIP memory model, which is why the mode stays opt-in and the default fold is
// a separate launch (pxa_tile_partials_fold); A/B numbers with the mode on depend on it.
// The RelError statistics of this launch, folded by the workgroup that finishes last (saves the fold launch
// of a stop check: ~3.4 us of device time plus a launch gap per step at stop_rate 1).  No fences: a
// device-scope release fence writes back the whole L2 of the XCD, per workgroup.  Instead every wavefront's
// lane 0 has written its (tile, wave) partials with relaxed device-scope atomic stores (wave_partials: write-
// through to the memory side) and waits for them to complete (s_waitcnt vmcnt(0)) before the workgroup counts
// itself with one relaxed device-scope atomic add; the last workgroup reads the partials with device-scope
// atomic loads (memory side again), folds each (statistic, row) in the order of pxa_tile_partials_fold
// (fold_tile_stat: same bits), writes the values and then, once they have completed, the completion flags to
// the host buffer with system-scope atomic stores, and resets the counter for the next launch.
template <typename T>
__device__ inline void tail_fold(const PgdParams<T>& p, const double* __restrict__ partials) {
  __shared__ double red[kThreads / 64];
  __shared__ unsigned last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores have completed
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(p.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (!last) return;
  auto ld = [](const double* a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  for (int64_t q = 0; q < 2 * p.fold_rows; ++q) {
    const int64_t stat = q / p.fold_rows, r = q - stat * p.fold_rows;
    const double t = fold_tile_stat(partials + 2 * r * p.fold_per_row + stat, p.fold_per_row, red, ld);
    if (threadIdx.x == 0) __hip_atomic_store(p.fold_vals + q, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store(p.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the values have reached host memory before the flags
    for (int64_t q = 0; q < 2 * p.fold_rows; ++q)
      __hip_atomic_store(p.fold_flags + q, p.fold_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The extra workgroup of a pxa_pgd_tv2d_plan_step_wpub launch: the previous launch's partials folded in the order of
// pxa_tile_partials_fold (fold_tile_stat: same sum order, same bits; the narrow load form, so that this branch adds
// no registers to the tile kernel's allocation), the values stored write-through to host memory
// (system-scope relaxed atomic stores), then -- once they have completed -- the flags.
template <typename T>
__device__ inline void publish_prev(const PgdParams<T>& p, double* red) {
  for (int64_t q = 0; q < 2 * p.fold_rows; ++q) {
    const int64_t stat = q / p.fold_rows, r = q - stat * p.fold_rows;
    const double t = fold_tile_stat<false>(p.pub_src + 2 * r * p.fold_per_row + stat, p.fold_per_row, red);
    if (threadIdx.x == 0) __hip_atomic_store(p.pub_vals + q, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the values have reached host memory before the flags
    for (int64_t q = 0; q < 2 * p.fold_rows; ++q)
      __hip_atomic_store(p.pub_flags + q, p.pub_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <typename T, int R>
__global__ void __launch_bounds__(kThreads, 4) pgd_tv2d_kernel(PgdParams<T> p, const T* __restrict__ x,
                                                            const T* __restrict__ xp, const T* __restrict__ b,
                                                            T* __restrict__ xn, double* __restrict__ partials) {
  using L = Layout<T, R>;
  // the publishing workgroup is block 0: dispatched in the first round, its fold is done long before the last tiles
  // (as the last block it ran beside the second round and could outlast it); the tile workgroups' index is shifted by
  // one, which rotates the XCD bands by one XCD and keeps each band on one XCD
  const unsigned pub = p.pub_src != nullptr ? 1u : 0u;
  if (pub && blockIdx.x == 0) {  // (no barrier shared with the tile workgroups)
    __shared__ double red[kThreads / 64];
    publish_prev<T>(p, red);
    return;
  }
  const unsigned vb = blockIdx.x - pub;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  if (kProbes && p.stagger && blockIdx.x < p.round1) {
    const unsigned sel = (unsigned)p.stagger >> 8, b = blockIdx.x >> 3;  // b: index within the XCD
    const bool late = sel == 1 ? (b & 1u) : sel == 2 ? ((b >> 1) & 1u) : sel == 3 ? ((b >> 2) & 1u) : ((b >> 5) & 1u);
    if (late)
      for (int i = 0; i < (p.stagger & 255); ++i) __builtin_amdgcn_s_sleep(16);
  }
  unsigned tile = xcd_tile(vb, p.ntiles);
  {  // the last XCD band walks backwards: an image's bottom-edge tiles (slower: boundary corrections)
     // are dispatched first instead of last, longest-first scheduling (2048^2: 29.2-29.3 -> 28.9-29.0 us)
    const unsigned nb = p.ntiles, q8 = nb >> 3, r8 = nb & 7u, g8 = vb & 7u;
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
  const T* xrs = (p.xref != nullptr ? p.xref : x) + (int64_t)s * img;
  // interior: the whole A window lies inside the image (so no boundary rows / columns of G either),
  // rows are 16-B aligned and 32-bit offsets suffice -> no bounds tests
  const bool interior = p.vec_ok && img <= 0x7fffffff && ty0 - 2 * R >= 0 && ty0 + TY + 2 * R <= p.n0 &&
                        tx0 - L::CA >= 0 && tx0 + TX + L::CA <= p.n1;
  if (interior)
    pgd_tile<T, R, false>(p, smem_raw, tile, ty0, tx0, xs, xps, bs, xns, partials, xrs);
  else
    pgd_tile<T, R, true>(p, smem_raw, tile, ty0, tx0, xs, xps, bs, xns, partials, xrs);
  if (p.fold_vals != nullptr) tail_fold<T>(p, partials);
}

thread_local int g_last_pgd_kernel = 0;  // pxa_pgd_tv2d_last_kernel

// ---- strip kernel: one workgroup walks a column strip of `slen` tiles downwards, keeping the window rows two
// vertically adjacent tiles share.  Tile i + 1's window (rows ty0 + TY - 2R .. ty0 + 2 TY + 2R) overlaps tile i's in
// 4R rows; only its TY new rows are loaded -- issued into registers while tile i computes (PXA_PGD_STRIP_ISSUE), so
// their latency overlaps pass B / the epilogue instead of opening the next tile -- then, once tile i's epilogue is
// done, the 4R shared rows move up in LDS (rows TY.. -> 0..) and the new rows are written below them as yk.  Per tile
// the arithmetic is the tile kernel's (same functions, same order): x_new and the RelError partials are bit-identical
// (tests/test_gpu_pgd_variants.py).  LDS: the tile carve + the TV-exchange area of waves 2, 3 (the tile kernel puts
// it in the window's bottom dead rows, which here are the next tile's top rows): 39.8 KB, four workgroups per CU.
// MEASURED SLOWER, kept opt-in for A/B (PXA_TUNE_PGD_KERNEL = strip length; round 6, profiles/r06b_pgd_strip_ab.txt):
// 2048^2 29.8 us against 23.9-25.2 (strips of 2), 4096^2 93.7 against 71.6 (8), C5 0.640 against 0.631 ms (16).  The
// prefetch can only be issued after the epilogue's own loads (held through pass B, the rows need ~24 VGPRs the
// passes do not have: 66 spilled), so it hides little; the loop keeps ~170 SGPRs of parameters and strip state live
// (spilled to VGPR lanes: a v_readlane before many tap uses in the sweeps); and the four workgroups of a CU walk their
// strips in lockstep for the whole launch, where the tile kernel's second round starts de-phased.  R 7, 8 spill VGPRs.
template <typename T, int R>
struct NewRows {  // the next tile's TY new window rows of x and x_prev, per thread
  using L = Layout<T, R>;
  static constexpr int NR = TY * L::NGA;
  static constexpr int K1 = cdiv(NR, kThreads);
  T xv[K1][L::V], pv[K1][L::V];
};

// Branch-free: every lane loads a whole 16-B vector from an address clamped into the image and zeroes it when the
// vector lies outside (the strip kernel runs only with vec_ok: rows 16-B aligned, n1 % V == 0, so a window vector is
// wholly inside or wholly outside) -- no exec-masked loads, whose results the compiler waited for and spilled.
template <typename T, int R>
__device__ inline void rows_issue(const PgdParams<T>& p, int ty0n, int tx0, const T* __restrict__ xs,
                                  const T* __restrict__ xps, NewRows<T, R>& w, const int lt) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
  const int n0 = p.n0, n1 = p.n1;
#pragma unroll
  for (int k = 0; k < NewRows<T, R>::K1; ++k) {
    int it = lt + k * kThreads;
    if (it >= NewRows<T, R>::NR) it = NewRows<T, R>::NR - 1;  // (surplus lanes of the last batch: dropped later)
    const int r = it / L::NGA, g = it - r * L::NGA;
    const int gr = ty0n + 2 * R + r, gc = tx0 - L::CA + V * g;  // window row 4R + r of the tile at ty0n
    const bool in = gr >= 0 && gr < n0 && gc >= 0 && gc < n1;
    const int cr = gr < 0 ? 0 : gr >= n0 ? n0 - 1 : gr, cc = gc < 0 ? 0 : gc >= n1 ? n1 - V : gc;
    const int64_t off = (int64_t)cr * n1 + cc;
    ld_vec<T, V>(xs + off, w.xv[k]);
    ld_vec<T, V>(xps + off, w.pv[k]);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      w.xv[k][v] = in ? w.xv[k][v] : T(0);
      w.pv[k][v] = in ? w.pv[k][v] : T(0);
    }
  }
}

// Next window, behind a barrier that follows every read of A by the current tile: the 4R rows shared with the next
// tile move up (rows TY .. TY + 4R - 1 -> 0 .. 4R - 1: disjoint ranges, so each thread copies its vectors directly),
// a barrier, then the new rows go in below them as yk (4R .. AR - 1, which overlaps the copy's source rows).
template <typename T, int R>
__device__ inline void window_advance(const PgdParams<T>& p, T* A, const NewRows<T, R>& w, const int lt) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
  using VT = typename Vec4<T>::type;
  constexpr int NS = 4 * R * L::NGA;
  VT* A4 = reinterpret_cast<VT*>(__builtin_assume_aligned(A, 16));
#pragma unroll
  for (int k = 0; k < cdiv(NS, kThreads); ++k) {
    const int it = lt + k * kThreads;
    if (it < NS) {
      const int r = it / L::NGA, g = it - r * L::NGA;
      A4[(r * L::AP) / V + g] = A4[((TY + r) * L::AP) / V + g];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NewRows<T, R>::K1; ++k) {
    const int it = lt + k * kThreads;
    if (it < NewRows<T, R>::NR) {
      const int r = it / L::NGA, g = it - r * L::NGA;
      T out[V];
#pragma unroll
      for (int v = 0; v < V; ++v) out[v] = fma(w.xv[k][v] - w.pv[k][v], p.a, w.xv[k][v]);  // as win_store
      st_vec<T, V>(A + (4 * R + r) * L::AP + V * g, out);
    }
  }
}

template <typename T, int R>
constexpr size_t kStripXOff = kGhOff<T, R> + kGhBytes<T, R>;  // the TV-exchange area of waves 2, 3
constexpr size_t kStripXBytes = (size_t)2 * kTvxFloats * sizeof(float);

template <typename T, int R>
__global__ void __launch_bounds__(kThreads, 4) pgd_strip_kernel(PgdParams<T> p, const T* __restrict__ x,
                                                             const T* __restrict__ xp, const T* __restrict__ b,
                                                             T* __restrict__ xn, double* __restrict__ partials) {
  using L = Layout<T, R>;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  T* A = reinterpret_cast<T*>(smem_raw);
  T* KT = A + L::AR * L::AP + L::AC * L::PTP;
  T* X23 = reinterpret_cast<T*>(smem_raw + kStripXOff<T, R>);
  const int tid = threadIdx.x;
  if (tid < 2 * R + 1) {
    KT[tid] = p.k0[tid];
    KT[kKT + tid] = p.k1[tid];
  }
  unsigned strip = xcd_tile(blockIdx.x, p.nstrips);
  {  // the last XCD band walks backwards (longest-first: the bottom-edge strips), as in the tile kernel
    const unsigned nb = p.nstrips, q8 = nb >> 3, r8 = nb & 7u, g8 = blockIdx.x & 7u;
    if (g8 == 7u) {
      const unsigned lo = 7u * q8 + (r8 < 7u ? r8 : 7u), len = q8 + (7u < r8 ? 1u : 0u);
      strip = lo + (len - 1u - (strip - lo));
    }
  }
  // strip = (image, strip group, tile column), tile column fastest: an XCD's band spans whole strip rows, so the
  // column halos of neighbouring strips are L2 hits
  const unsigned tiles1 = (unsigned)p.tiles1, per_img = p.sgroups * tiles1;
  const unsigned si = strip / per_img, rem = strip - si * per_img;
  const unsigned sg = rem / tiles1, tc = rem - sg * tiles1;
  const int tr0 = (int)(sg * p.slen);
  const int tr1 = tr0 + (int)p.slen < p.tiles0 ? tr0 + (int)p.slen : p.tiles0;
  const int tx0 = (int)tc * TX;
  const int64_t img = (int64_t)p.n0 * p.n1;
  const T* xs = x + (int64_t)si * img;
  const T* xps = xp + (int64_t)si * img;
  const T* bs = b + (int64_t)(si % (unsigned)p.y_images) * img;
  T* xns = xn + (int64_t)si * img;
  const T* xrs = (p.xref != nullptr ? p.xref : x) + (int64_t)si * img;
  const unsigned tpi = (unsigned)p.tiles0 * tiles1;
  const bool cols_in = p.vec_ok && img <= 0x7fffffff && tx0 - L::CA >= 0 && tx0 + TX + L::CA <= p.n1;
  {
    const int ty0 = tr0 * TY;
#if PXA_PGD_PRIO
    __builtin_amdgcn_s_setprio(PXA_PGD_PRIO);
#endif
    if (cols_in && ty0 - 2 * R >= 0 && ty0 + TY + 2 * R <= p.n0) load_window<T, R, false>(p, A, ty0, tx0, xs, xps);
    else load_window<T, R, true>(p, A, ty0, tx0, xs, xps);
#if PXA_PGD_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  }
  NewRows<T, R> nw;
  for (int tr = tr0; tr < tr1; ++tr) {
    // the thread index laundered per tile: its derived addresses are recomputed in every tile instead of being
    // hoisted out of the loop and kept live across it (the loop-invariant form spilled ~70-200 VGPRs)
    int ltid = tid;
    asm volatile("" : "+v"(ltid));
    const int ty0 = tr * TY;
    const unsigned tile = si * tpi + (unsigned)tr * tiles1 + tc;
    const bool more = tr + 1 < tr1;
    __syncthreads();  // the window of this tile is in A
    // (issued for the last tile of the strip too, clamped into the image, so that no branch guards the loads)
    auto issue = [&]() { rows_issue<T, R>(p, ty0 + TY, tx0, xs, xps, nw, ltid); };
    if (cols_in && ty0 - 2 * R >= 0 && ty0 + TY + 2 * R <= p.n0)
      pgd_tile_body<T, R, false, PXA_PGD_STRIP_DEPTH, false>(p, smem_raw, tile, ty0, tx0, bs, xns, partials, xrs, X23, issue, ltid);
    else
      pgd_tile_body<T, R, true, PXA_PGD_STRIP_DEPTH, false>(p, smem_raw, tile, ty0, tx0, bs, xns, partials, xrs, X23, issue, ltid);
    if (more) {
      __syncthreads();  // every read of this window is done
      window_advance<T, R>(p, A, nw, ltid);
    }
  }
  if (p.fold_vals != nullptr) tail_fold<T>(p, partials);
}

template <typename T, int R>
int launch_pgd_strip(const PgdParams<T>& p, const void* x, const void* xp, const void* b, void* xn, double* partials,
                     hipStream_t s) {
  const size_t smem = kStripXOff<T, R> + kStripXBytes;
  auto kern = pgd_strip_kernel<T, R>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(p.nstrips), dim3(kThreads), smem, s, p, (const T*)x, (const T*)xp, (const T*)b,
                     (T*)xn, partials);
  return last_launch_status();
}

// ---- pipelined kernel (PXA_TUNE_PGD_KERNEL = -1): a resident grid of two workgroups per CU, each walking the tiles of
// its XCD's band (i = blockIdx.x, + grid, ...: the same XCD every time).  The raw x / x_prev window of the NEXT tile is
// fetched by LDS-DMA (global_load_lds_dwordx4: no VGPR destination, so nothing is held through the passes) into a
// staging area beside the tile carve while the current tile runs passes A / B and its epilogue; then one pass turns
// the staged window into yk in A (win_store's arithmetic: the same bits as the tile kernel's phase 0).  The body
// uses raw barriers (body_sync<true>) so that the fetch stays in flight through them.  LDS: carve 36.4 KB + staging
// 40 KB = 75.5 KB per workgroup (fp32, R = 6), two per CU; edge tiles are fetched with clamped addresses and their
// outside vectors zeroed (vec_ok: a 16-B vector lies wholly inside or outside the image).
template <typename T, int R>
constexpr int kPipeChunks = cdiv(Layout<T, R>::N0, 64);  // one LDS-DMA wave-instruction = 64 window vectors
template <typename T, int R>
constexpr size_t kPipeArr = (size_t)kPipeChunks<T, R> * 64 * 16;  // bytes of one staged window array
template <typename T, int R>
constexpr size_t kPipeRawOff = (kGhOff<T, R> + kGhBytes<T, R> + 15) / 16 * 16;
template <typename T, int R>
constexpr size_t kPipeBytes = kPipeRawOff<T, R> + 2 * kPipeArr<T, R>;

template <typename T, int R>
__device__ inline void pipe_issue(const PgdParams<T>& p, unsigned char* raw, int ty0, int tx0, const T* __restrict__ xs,
                                  const T* __restrict__ xps, const int tid) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
  constexpr int NW = kThreads / 64;
  static_assert(V * sizeof(T) == 16, "one 16-B vector per lane");
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int n0 = p.n0, n1 = p.n1;
#pragma unroll
  for (int k = 0; k < cdiv(kPipeChunks<T, R>, NW); ++k) {
    const int c = wv + NW * k;
    if (c < kPipeChunks<T, R>) {
      int it = c * 64 + lane;
      if (it >= L::N0) it = L::N0 - 1;  // (the last piece's surplus lanes fill the staging padding)
      int r, g;
      win_rg<T, R>(it, r, g);
      int gr = ty0 - 2 * R + r, gc = tx0 - L::CA + V * g;
      gr = gr < 0 ? 0 : gr >= n0 ? n0 - 1 : gr;
      gc = gc < 0 ? 0 : gc > n1 - V ? n1 - V : gc;
      const int64_t off = (int64_t)gr * n1 + gc;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(xs + off),
                                       (__attribute__((address_space(3))) void*)(raw + (size_t)c * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(xps + off),
                                       (__attribute__((address_space(3))) void*)(raw + kPipeArr<T, R> + (size_t)c * 1024),
                                       16, 0, 0);
    }
  }
}

// staged window -> yk in A (and the window partials), behind a barrier after every wave's pieces have landed
template <typename T, int R>
__device__ inline void pipe_window(const PgdParams<T>& p, T* A, const unsigned char* raw, int ty0, int tx0,
                                   double* __restrict__ partials, unsigned tile, const int tid) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
  const int n0 = p.n0, n1 = p.n1;
  const T* rx = reinterpret_cast<const T*>(raw);
  const T* rp = reinterpret_cast<const T*>(raw + kPipeArr<T, R>);
  Window<T, R> w;
#pragma unroll
  for (int k = 0; k < Window<T, R>::K0; ++k) {
    const int it = tid + k * kThreads;
    if (it < L::N0) {
      int r, g;
      win_rg<T, R>(it, r, g);
      const int gr = ty0 - 2 * R + r, gc = tx0 - L::CA + V * g;
      ld_vec<T, V>(rx + V * it, w.xv[k]);
      ld_vec<T, V>(rp + V * it, w.pv[k]);
      if (!(gr >= 0 && gr < n0 && gc >= 0 && gc < n1)) {
#pragma unroll
        for (int v = 0; v < V; ++v) w.xv[k][v] = w.pv[k][v] = T(0);
      }
    }
  }
  win_store<T, R>(p, A, w, tid);
  if (p.win_part && partials != nullptr) win_partials<T, R>(w, partials, tile, tid);
}

template <typename T, int R>
__global__ void __launch_bounds__(kThreads, 2) pgd_pipe_kernel(PgdParams<T> p, const T* __restrict__ x,
                                                            const T* __restrict__ xp, const T* __restrict__ b,
                                                            T* __restrict__ xn, double* __restrict__ partials) {
  using L = Layout<T, R>;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const unsigned nw = p.pipe_wgs;
  if (p.pub_src != nullptr && blockIdx.x == nw) {  // the publishing workgroup (its reduction area: the carve's start)
    publish_prev<T>(p, reinterpret_cast<double*>(smem_raw));
    return;
  }
  T* A = reinterpret_cast<T*>(smem_raw);
  T* KT = A + L::AR * L::AP + L::AC * L::PTP;
  unsigned char* raw = smem_raw + kPipeRawOff<T, R>;
  const int tid = threadIdx.x;
  if (tid < 2 * R + 1) {
    KT[tid] = p.k0[tid];
    KT[kKT + tid] = p.k1[tid];
  }
  const unsigned tpi = (unsigned)p.tiles0 * (unsigned)p.tiles1;
  const int64_t img = (int64_t)p.n0 * p.n1;
  // virtual block index -> (tile, image, tile origin), as the tile kernel maps its block index (XCD band, the last
  // band backwards)
  auto locate = [&](unsigned i, unsigned& tile, unsigned& si, int& ty0, int& tx0) {
    tile = xcd_tile(i, p.ntiles);
    const unsigned nb = p.ntiles, q8 = nb >> 3, r8 = nb & 7u, g8 = i & 7u;
    if (g8 == 7u) {
      const unsigned lo = 7u * q8 + (r8 < 7u ? r8 : 7u), len = q8 + (7u < r8 ? 1u : 0u);
      tile = lo + (len - 1u - (tile - lo));
    }
    si = tile / tpi;
    const unsigned tr = tile - si * tpi, trow = tr / (unsigned)p.tiles1;
    ty0 = (int)trow * TY;
    tx0 = (int)(tr - trow * (unsigned)p.tiles1) * TX;
  };
  unsigned i = blockIdx.x, tile, si;
  int ty0, tx0;
  locate(i, tile, si, ty0, tx0);
  pipe_issue<T, R>(p, raw, ty0, tx0, x + (int64_t)si * img, xp + (int64_t)si * img, tid);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  body_sync<true>();
  pipe_window<T, R>(p, A, raw, ty0, tx0, partials, tile, tid);
  using KP = const __attribute__((address_space(4))) PgdParams<T>*;
  for (;;) {
    // the parameters re-read (scalar loads from the kernel-argument segment) per tile: hoisted out of the loop, the
    // taps and geometry stay live across it and spill
    KP kp = (KP)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    const PgdParams<T>& p = *(const PgdParams<T>*)kp;
    body_sync<true>();  // A holds this tile's window; the staging area is free
    const unsigned inext = i + nw;
    const bool more = inext < p.ntiles;
    unsigned tile_n = 0, si_n = 0;
    int ty0n = 0, tx0n = 0;
    if (more) {
      locate(inext, tile_n, si_n, ty0n, tx0n);
      pipe_issue<T, R>(p, raw, ty0n, tx0n, x + (int64_t)si_n * img, xp + (int64_t)si_n * img, tid);
    }
    const T* bs = b + (int64_t)(si % (unsigned)p.y_images) * img;
    T* xns = xn + (int64_t)si * img;
    const T* xrs = (p.xref != nullptr ? p.xref : x) + (int64_t)si * img;
    const bool interior = img <= 0x7fffffff && ty0 - 2 * R >= 0 && ty0 + TY + 2 * R <= p.n0 && tx0 - L::CA >= 0 &&
                          tx0 + TX + L::CA <= p.n1;
    double* bp = p.win_part ? nullptr : partials;
    if (interior)
      pgd_tile_body<T, R, false, PXA_PGD_SWEEP_DEPTH, true>(p, smem_raw, tile, ty0, tx0, bs, xns, bp, xrs, nullptr,
                                                            NoHook{}, tid);
    else
      pgd_tile_body<T, R, true, PXA_PGD_SWEEP_DEPTH, true>(p, smem_raw, tile, ty0, tx0, bs, xns, bp, xrs, nullptr,
                                                           NoHook{}, tid);
    if (!more) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of the next window have landed
    body_sync<true>();                                 // ... every wave's, and every read of A by this tile is done
    pipe_window<T, R>(p, A, raw, ty0n, tx0n, partials, tile_n, tid);
    i = inext;
    tile = tile_n;
    si = si_n;
    ty0 = ty0n;
    tx0 = tx0n;
  }
}

// resident workgroups per CU of the pipelined kernel, and the CU count of the current device (cached per device)
constexpr int kPipePerCu = 2;
inline int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

template <typename T, int R>
int launch_pgd_pipe(const PgdParams<T>& p, const void* x, const void* xp, const void* b, void* xn, double* partials,
                    hipStream_t s) {
  const size_t smem = kPipeBytes<T, R>;
  auto kern = pgd_pipe_kernel<T, R>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(p.pipe_wgs + (p.pub_src != nullptr ? 1u : 0u)), dim3(kThreads), smem, s, p, (const T*)x,
                     (const T*)xp, (const T*)b, (T*)xn, partials);
  return last_launch_status();
}

template <typename T, int R>
int launch_pgd(const PgdParams<T>& p, const void* x, const void* xp, const void* b, void* xn, double* partials,
               hipStream_t s) {
  constexpr bool strip_fits = kStripXOff<T, R> + kStripXBytes <= (size_t)160 * 1024;  // (fp64 at large R: no)
  constexpr bool pipe_fits = sizeof(T) == 4 && kPipeBytes<T, R> * kPipePerCu <= (size_t)160 * 1024;
  if (pipe_fits && p.pipe_wgs > 0) {
    const int e = launch_pgd_pipe<T, R>(p, x, xp, b, xn, partials, s);
    if (e == PXA_OK) g_last_pgd_kernel = 3;
    return e;
  }
  if (strip_fits && p.slen >= 2) {
    const int e = launch_pgd_strip<T, R>(p, x, xp, b, xn, partials, s);
    if (e == PXA_OK) g_last_pgd_kernel = 2;
    return e;
  }
  g_last_pgd_kernel = 1;
  // Layout + the ghost terms (+ the timing trace under PXA_TUNE_PGD_DIAG bit 5)
  const size_t smem = kGhOff<T, R> + kGhBytes<T, R> + ((p.diag & 32) ? 256 : 0);
  auto kern = pgd_tv2d_kernel<T, R>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(kGhOff<T, R> + kGhBytes<T, R> + 256));
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(p.ntiles + (p.pub_src != nullptr ? 1u : 0u)), dim3(kThreads), smem, s, p, (const T*)x,
                     (const T*)xp, (const T*)b, (T*)xn, partials);
  return last_launch_status();
}


// Iteration-invariant parameters (taps folded per offset, G = k (*) k, geometry, prox kind); `R` the blur reach.
template <typename T>
int pgd_params(int64_t stack, int64_t y_images, int64_t n0, int64_t n1, int nt0, const int32_t* off0,
               const double* coef0, int nt1, const int32_t* off1, const double* coef1, double h0, double h1, double lam,
               double mu, int prox, PgdParams<T>& p, int& R) {
  PXA_CHECK_ARG(stack >= 1 && n0 >= 1 && n1 >= 1 && y_images >= 1 && stack % y_images == 0);
  PXA_CHECK_ARG(n0 <= 0x7fffffff && n1 <= 0x7fffffff);
  PXA_CHECK_ARG(prox >= 0 && prox <= 2);
  PXA_CHECK_ARG(nt0 >= 1 && nt1 >= 1 && off0 && off1 && coef0 && coef1);
  R = 1;  // TV needs a 1-pixel halo even for a 1-tap blur
  for (int q = 0; q < nt0; ++q) R = abs(off0[q]) > R ? abs(off0[q]) : R;
  for (int q = 0; q < nt1; ++q) R = abs(off1[q]) > R ? abs(off1[q]) : R;
  if (R > kMaxR) return PXA_ERR_UNSUPPORTED;
  p = PgdParams<T>{};
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
  p.tv = lam != 0.0;
  p.prox = prox;
  p.round1 = 4u * 256u;
  return PXA_OK;
}

// One launch from prepared parameters: the per-step scalars and arrays, then the kernel of reach R.
template <typename T>
int pgd_run(PgdParams<T> p, int R, double a, double tau, double prox_w, const void* x, const void* x_prev,
            const void* hty, void* x_new, double* partials, const void* x_ref, double* rel_values, uint32_t* rel_flags,
            uint32_t seq, unsigned* counter, hipStream_t s, int win_part = 0, const double* pub_src = nullptr,
            double* pub_vals = nullptr, uint32_t* pub_flags = nullptr, uint32_t pub_seq = 0) {
  PXA_CHECK_ARG(x && x_prev && hty && x_new);
  PXA_CHECK_ARG(x_new != x && x_new != x_prev && x_new != x_ref);
  PXA_CHECK_ARG(rel_values == nullptr || (partials != nullptr && rel_flags != nullptr && counter != nullptr));
  p.a = (T)a;
  p.tau = (T)tau;
  p.pw = (T)prox_w;
  constexpr int V = kVecN<T>;
  p.vec_ok = (p.n1 % V == 0) && aligned16(x) && aligned16(x_prev) && aligned16(hty) && aligned16(x_new) &&
             (x_ref == nullptr || aligned16(x_ref));
  p.xref = (partials != nullptr && x_ref != nullptr && x_ref != x) ? (const T*)x_ref : nullptr;
  p.diag = kProbes ? tuning(PXA_TUNE_PGD_DIAG) : 0;
  p.stagger = kProbes ? tuning(PXA_TUNE_PGD_STAGGER) : 0;
  p.fold_vals = rel_values;
  p.fold_flags = (unsigned*)rel_flags;
  p.fold_seq = (unsigned)seq;
  p.counter = counter;
  // rows of the RelError statistics = rows of the solver state: y_images images each (batch-as-axis); the
  // slots of one image, hence of one row, are contiguous
  p.fold_rows = p.stack / p.y_images;
  p.fold_per_row = (int64_t)p.ntiles * (kThreads / 64) / p.fold_rows;
  p.win_part = win_part;
  PXA_CHECK_ARG(!win_part || (partials != nullptr && rel_values == nullptr));
  PXA_CHECK_ARG(pub_src == nullptr || (pub_vals != nullptr && pub_flags != nullptr && pub_src != partials));
  p.pub_src = pub_src;
  p.pub_vals = pub_vals;
  p.pub_flags = (unsigned*)pub_flags;
  p.pub_seq = (unsigned)pub_seq;
  // kernel choice (PXA_TUNE_PGD_KERNEL): 0 / 1 the tile kernel (default); v >= 2 the strip kernel with strips of v
  // tiles (A/B and tests: measured slower, see the strip kernel's comment)
  {
    const int64_t kv = tuning(PXA_TUNE_PGD_KERNEL);
    int64_t sl = 1;
    if (kv >= 2) sl = kv;
    if (sl > p.tiles0) sl = p.tiles0;
    if (sl < 1 || !p.vec_ok) sl = 1;  // (the strip kernel's row prefetch moves whole 16-B vectors only)
    p.slen = (unsigned)sl;
    p.sgroups = (unsigned)((p.tiles0 + sl - 1) / sl);
    const int64_t ns = p.stack * (int64_t)p.sgroups * p.tiles1;
    p.nstrips = (unsigned)ns;
    if (ns > 0x7fffffff || win_part || pub_src) p.slen = 1;  // (window partials / publication: the tile kernel)
    // PXA_TUNE_PGD_PIPE = 1: the pipelined kernel (whole 16-B vectors only; not with the last-workgroup fold)
    p.pipe_wgs = 0;
    if (tuning(PXA_TUNE_PGD_PIPE) == 1 && p.vec_ok && rel_values == nullptr) {
      const unsigned cap = (unsigned)(kPipePerCu * device_cus());
      unsigned nw = p.ntiles < cap ? p.ntiles : cap;
      if (nw >= 8) nw -= nw % 8;  // a multiple of 8: every workgroup stays on its XCD's band
      p.pipe_wgs = nw;
      p.slen = 1;
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
  return st;
}

template <typename T>
int pgd_entry(int64_t stack, int64_t y_images, int64_t n0, int64_t n1, int nt0, const int32_t* off0,
              const double* coef0, int nt1, const int32_t* off1, const double* coef1, double h0, double h1, double lam,
              double mu, double a, double tau, int prox, double prox_w, const void* x, const void* x_prev,
              const void* hty, void* x_new, double* partials, const void* x_ref, hipStream_t s) {
  PgdParams<T> p;
  int R = 1;
  const int e = pgd_params<T>(stack, y_images, n0, n1, nt0, off0, coef0, nt1, off1, coef1, h0, h1, lam, mu, prox, p, R);
  if (e != PXA_OK) return e;
  return pgd_run<T>(p, R, a, tau, prox_w, x, x_prev, hty, x_new, partials, x_ref, nullptr, nullptr, 0, nullptr, s);
}

// pxa_pgd_tv2d_plan: the prepared parameters of one problem (both precisions' storage, one used) and the
// device counter of the last-workgroup fold
struct PgdPlan {
  int dtype;
  int R;
  PgdParams<float> pf;
  PgdParams<double> pd;
  unsigned* counter;
};

}  // namespace
}  // namespace pxa

using namespace pxa;

extern "C" {

int pxa_pgd_tv2d_last_kernel(void) { return g_last_pgd_kernel; }

int pxa_pgd_tile_trace(uint64_t* host_out, int n) {
  if (!kProbes) return PXA_ERR_UNSUPPORTED;  // the phase trace exists only in the probe build
  if (!host_out || n < 0 || n > kTraceWords) return PXA_ERR_ARG;
  if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_tile_trace), (size_t)n * 8, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return PXA_ERR_UNSUPPORTED;
  return PXA_OK;
}

int pxa_pgd_tv2d_partials_count(int64_t stack, int64_t n0, int64_t n1) {
  int64_t t = stack * ((n0 + TY - 1) / TY) * ((n1 + TX - 1) / TX) * kPartWaves;
  return (int)t;
}

int pxa_pgd_tv2d_plan(int dtype, int64_t stack, int64_t y_images, int64_t n0, int64_t n1, int nt0, const int32_t* off0,
                      const double* coef0, int nt1, const int32_t* off1, const double* coef1, double h0, double h1,
                      double lam, double mu, int prox, void** plan) {
  PXA_CHECK_ARG(plan != nullptr);
  *plan = nullptr;
  PgdPlan* pl = new PgdPlan();
  pl->dtype = dtype;
  int e = PXA_ERR_DTYPE;
  if (dtype == PXA_F32)
    e = pgd_params<float>(stack, y_images, n0, n1, nt0, off0, coef0, nt1, off1, coef1, h0, h1, lam, mu, prox, pl->pf, pl->R);
  else if (dtype == PXA_F64)
    e = pgd_params<double>(stack, y_images, n0, n1, nt0, off0, coef0, nt1, off1, coef1, h0, h1, lam, mu, prox, pl->pd, pl->R);
  if (e == PXA_OK) {  // HIP failures: the positive hipError_t (the header's convention: HIP codes > 0, PXA_ERR_* < 0)
    hipError_t he = hipMalloc((void**)&pl->counter, sizeof(unsigned));
    if (he != hipSuccess) pl->counter = nullptr;
    else he = hipMemset(pl->counter, 0, sizeof(unsigned));
    if (he != hipSuccess) e = (int)he > 0 ? (int)he : PXA_ERR_UNSUPPORTED;
  }
  if (e != PXA_OK) {
    if (pl->counter) (void)hipFree(pl->counter);
    delete pl;
    return e;
  }
  *plan = pl;
  return PXA_OK;
}

int pxa_pgd_tv2d_plan_step(void* plan, double a, double tau, double prox_w, const void* x, const void* x_prev,
                           const void* hty, void* x_new, double* partials, const void* x_ref, double* rel_values,
                           uint32_t* rel_flags, uint32_t seq, void* stream) {
  PXA_CHECK_ARG(plan != nullptr);
  const PgdPlan* pl = (const PgdPlan*)plan;
  if (pl->dtype == PXA_F32)
    return pgd_run<float>(pl->pf, pl->R, a, tau, prox_w, x, x_prev, hty, x_new, partials, x_ref, rel_values, rel_flags,
                          seq, pl->counter, as_stream(stream));
  return pgd_run<double>(pl->pd, pl->R, a, tau, prox_w, x, x_prev, hty, x_new, partials, x_ref, rel_values, rel_flags, seq,
                         pl->counter, as_stream(stream));
}

int pxa_pgd_tv2d_plan_step_fold(void* plan, double a, double tau, double prox_w, const void* x, const void* x_prev,
                                const void* hty, void* x_new, double* partials, const void* x_ref, double* rel_values,
                                uint32_t* rel_flags, uint32_t seq, void* stream) {
  PXA_CHECK_ARG(plan != nullptr && partials != nullptr && rel_values != nullptr && rel_flags != nullptr);
  const PgdPlan* pl = (const PgdPlan*)plan;
  const int64_t stack = pl->dtype == PXA_F32 ? pl->pf.stack : pl->pd.stack;
  const int64_t rows = stack / (pl->dtype == PXA_F32 ? pl->pf.y_images : pl->pd.y_images);
  const int64_t per_row = (int64_t)(pl->dtype == PXA_F32 ? pl->pf.ntiles : pl->pd.ntiles) * (kThreads / 64) / rows;
  const int e = pxa_pgd_tv2d_plan_step(plan, a, tau, prox_w, x, x_prev, hty, x_new, partials, x_ref, nullptr, nullptr,
                                       0, stream);
  if (e != PXA_OK) return e;
  return pxa_tile_partials_fold(rows, per_row, partials, rel_values, rel_flags, seq, stream);
}

int pxa_pgd_tv2d_plan_step_wfold(void* plan, double a, double tau, double prox_w, const void* x, const void* x_prev,
                                 const void* hty, void* x_new, double* partials, double* rel_values, uint32_t* rel_flags,
                                 uint32_t seq, void* stream) {
  PXA_CHECK_ARG(plan != nullptr && partials != nullptr && rel_values != nullptr && rel_flags != nullptr);
  const PgdPlan* pl = (const PgdPlan*)plan;
  const int64_t stack = pl->dtype == PXA_F32 ? pl->pf.stack : pl->pd.stack;
  const int64_t rows = stack / (pl->dtype == PXA_F32 ? pl->pf.y_images : pl->pd.y_images);
  const int64_t per_row = (int64_t)(pl->dtype == PXA_F32 ? pl->pf.ntiles : pl->pd.ntiles) * (kThreads / 64) / rows;
  int e;
  if (pl->dtype == PXA_F32)
    e = pgd_run<float>(pl->pf, pl->R, a, tau, prox_w, x, x_prev, hty, x_new, partials, nullptr, nullptr, nullptr, 0,
                       pl->counter, as_stream(stream), 1);
  else
    e = pgd_run<double>(pl->pd, pl->R, a, tau, prox_w, x, x_prev, hty, x_new, partials, nullptr, nullptr, nullptr, 0,
                        pl->counter, as_stream(stream), 1);
  if (e != PXA_OK) return e;
  return pxa_tile_partials_fold(rows, per_row, partials, rel_values, rel_flags, seq, stream);
}

int pxa_pgd_tv2d_plan_step_wpub(void* plan, double a, double tau, double prox_w, const void* x, const void* x_prev,
                                const void* hty, void* x_new, double* partials, const double* prev_partials,
                                double* rel_values, uint32_t* rel_flags, uint32_t seq, void* stream) {
  PXA_CHECK_ARG(plan != nullptr && partials != nullptr);
  PXA_CHECK_ARG(prev_partials == nullptr || (rel_values != nullptr && rel_flags != nullptr));
  const PgdPlan* pl = (const PgdPlan*)plan;
  if (pl->dtype == PXA_F32)
    return pgd_run<float>(pl->pf, pl->R, a, tau, prox_w, x, x_prev, hty, x_new, partials, nullptr, nullptr, nullptr, 0,
                          pl->counter, as_stream(stream), 1, prev_partials, rel_values, rel_flags, seq);
  return pgd_run<double>(pl->pd, pl->R, a, tau, prox_w, x, x_prev, hty, x_new, partials, nullptr, nullptr, nullptr, 0,
                         pl->counter, as_stream(stream), 1, prev_partials, rel_values, rel_flags, seq);
}

int pxa_pgd_tv2d_plan_free(void* plan) {
  if (plan == nullptr) return PXA_OK;
  PgdPlan* pl = (PgdPlan*)plan;
  if (pl->counter) (void)hipFree(pl->counter);
  delete pl;
  return PXA_OK;
}

int pxa_pgd_tv2d_step(int dtype, int64_t stack, int64_t y_images, int64_t n0, int64_t n1, int nt0, const int32_t* off0,
                      const double* coef0, int nt1, const int32_t* off1, const double* coef1, double h0, double h1,
                      double lam, double mu, double a, double tau, int prox, double prox_w, const void* x,
                      const void* x_prev, const void* hty, void* x_new, double* partials, const void* x_ref,
                      void* stream) {
  PXA_DISPATCH(dtype, T,
               return pgd_entry<T>(stack, y_images, n0, n1, nt0, off0, coef0, nt1, off1, coef1, h0, h1, lam, mu, a,
                                   tau, prox, prox_w, x, x_prev, hty, x_new, partials, x_ref, as_stream(stream)));
}

}  // extern "C"
