// Kernels A (axis-0 march) and B (in-plane G12 + point-wise update) of the fused PD3O / Condat-Vu
// step; see pds3d.hip for the algorithm.  Instantiated per dtype in pds_{a,b}_{f32,f64}.hip so that
// the build compiles them in parallel.
#pragma once
#include <type_traits>

#include "tile2d.hpp"

namespace pxa {
namespace pds {

using namespace tile2d;

constexpr int kMaxR0 = 8;
constexpr int kAThreads = 256;

template <int I, int N, typename F>
__device__ inline void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// Volume geometry shared by the kernels.  `stack` volumes of n0 x n1 x n2 (n0 = 1 for 2-D images);
// z holds D direction fields per volume, direction-major: direction d differentiates axis d + 3 - D.
template <typename T>
struct PdsGeom {
  int64_t stack, y_images;
  int n0, n1, n2, D;
  T c0[3], c1[3];  // forward-difference taps per AXIS: (K x)_a[i] = c0 x[i] + c1 x[i + e_a]
};

template <typename T, int NP>
__device__ inline void ldn(const T* p, T (&v)[NP]) {
  if constexpr (NP == 2) {
    if constexpr (sizeof(T) == 4) {
      const float2 t = *reinterpret_cast<const float2*>(p);
      v[0] = t.x;
      v[1] = t.y;
    } else {
      const double2 t = *reinterpret_cast<const double2*>(p);
      v[0] = t.x;
      v[1] = t.y;
    }
  } else {
    v[0] = p[0];
  }
}
template <typename T, int NP>
__device__ inline void stn(T* p, const T (&v)[NP]) {
  if constexpr (NP == 2) {
    if constexpr (sizeof(T) == 4)
      *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
    else
      *reinterpret_cast<double2*>(p) = make_double2(v[0], v[1]);
  } else {
    p[0] = v[0];
  }
}

// Non-temporal (streaming) forms of ldn / stn for arrays a kernel reads or writes exactly once: they do not
// displace the re-read neighbour rows (w at row + 1 / row - 1) from the XCD's 4 MB L2, which 128 marching
// workgroups per XCD otherwise turn over within about one plane.
template <typename T, int NP>
__device__ inline void ldn_nt(const T* p, T (&v)[NP]) {
  if constexpr (NP == 1) {
    v[0] = __builtin_nontemporal_load(p);
  } else {
    typedef T vt __attribute__((ext_vector_type(NP)));
    const vt r = __builtin_nontemporal_load(reinterpret_cast<const vt*>(p));
#pragma unroll
    for (int i = 0; i < NP; ++i) v[i] = r[i];
  }
}
template <typename T, int NP>
__device__ inline void stn_nt(T* p, const T (&v)[NP]) {
  if constexpr (NP == 1) {
    __builtin_nontemporal_store(v[0], p);
  } else {
    typedef T vt __attribute__((ext_vector_type(NP)));
    vt r;
#pragma unroll
    for (int i = 0; i < NP; ++i) r[i] = v[i];
    __builtin_nontemporal_store(r, reinterpret_cast<vt*>(p));
  }
}

// ------------------------------------------------------------------ dual update of one position
// z_new = relax(fenchel_prox_h(z + sigma K w)) for the directions a_first..2 of one position; kernels C
// and D both go through these helpers, so the three-launch and the look-ahead steps produce the same bits.
template <typename T>
__device__ inline T dual_in(T zc, T wc, T wn, T c0, T c1, T sigma) {
  const T kw = fma(c0, wc, c1 * wn);  // forward difference (pxa_gradient2)
  return fma(sigma, kw, zc);          // z + sigma K w
}

// one direction's term of K^T z at a position: the flipped 2-tap adjoint c1 z[i - e_a] + c0 z[i]
// (pxa_gradient2_adjoint).  Explicit fmas here and in the dual helpers: every kernel that evaluates these
// expressions (A, B, C, D, in whatever inlined context) rounds them the same way.
template <typename T>
__device__ inline T kt_term(T c1, T zm, T c0, T zc) {
  return fma(c1, zm, c0 * zc);
}

// fenchel_prox_{sigma h}(zin) for h = lam L1 / lam L21 (operator.py:905-944 evaluates the Moreau form
// zin - sigma prox_{h / sigma}(zin / sigma)), evaluated as what that form equals: the projection onto the
// dual-norm ball of radius lam (L1: the box [-lam, lam] per direction; L21: the l2 ball over the
// directions).  Same value up to rounding, without the three fp32 divisions per position the Moreau form
// costs (the fused kernels are VALU-heavy).  Then the relaxation (PD3O: (1 - rho) z + rho z_t; Condat-Vu:
// rho z_t + (1 - rho) z).
template <typename T, bool ISO, bool PD3O>
__device__ inline void dual_out(const T (&zc)[3], const T (&zin)[3], int a_first, T lam, T rho, T omr, T (&zn)[3]) {
  T zt[3];
  if constexpr (ISO) {
    T ss = T(0);
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
      if (ax < a_first) continue;
      ss = fma(zin[ax], zin[ax], ss);
    }
    const T nrm = sqrt(ss);
    const T f = nrm > lam ? lam / nrm : T(1);
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) zt[ax] = zin[ax] * f;
  } else {
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) zt[ax] = fmin(fmax(zin[ax], -lam), lam);
  }
#pragma unroll
  for (int ax = 0; ax < 3; ++ax)
    zn[ax] = ax < a_first ? T(0) : (PD3O ? fma(omr, zc[ax], rho * zt[ax]) : fma(rho, zt[ax], omr * zc[ax]));
}

// ------------------------------------------------------------------ kernel A: axis-0 march
template <typename T>
struct PdsA {
  PdsGeom<T> g;
  T k0[2 * kMaxR0 + 1];  // axis-0 taps, dense window t = -R0..R0
  T tau, pw;
  int prox;
  int seg;  // planes per segment (grid.y splits axis 0 into segments)
};

// Thread = NP consecutive in-plane positions of one volume; it walks planes [pb - 2 R0, pe + 2 R0)
// and outputs Q = G0 v on planes [pb, pe) (R0 > 0).  v = x (Condat-Vu) or prox_g(u - tau K^T z) (PD3O,
// stored to xo on [pb, pe)).
template <typename T, int R0, int NP, bool PD3O>
__global__ void __launch_bounds__(kAThreads) pds_axis0_kernel(PdsA<T> p, const T* __restrict__ src,
                                                              const T* __restrict__ z, T* __restrict__ xo,
                                                              T* __restrict__ q) {
  constexpr int RING = 2 * R0 + 1;
  // kernel arguments are copied to registers: the lambdas below capture by reference, and taking the
  // address of a kernel argument would move the whole parameter block to scratch memory
  const PdsGeom<T> g = p.g;
  const T tau = p.tau, pw = p.pw;
  const int prox = p.prox;
  T k0[RING];
#pragma unroll
  for (int t = 0; t < RING; ++t) k0[t] = p.k0[t];
  const int64_t M = (int64_t)g.n1 * g.n2;
  // XCD-banded block index: the row-1 neighbour of K^T z is usually read from the same XCD's L2
  const int64_t j0 = ((int64_t)xcd_tile(blockIdx.x, gridDim.x) * kAThreads + threadIdx.x) * NP;
  if (j0 >= M) return;  // no barriers below
  const int64_t s = blockIdx.z;
  const int64_t N = M * g.n0;
  const int row = (int)(j0 / g.n2), col = (int)(j0 - (int64_t)row * g.n2);
  const T* in = src + s * N + j0;
  const T* zs = z + s * g.D * N + j0;
  T* xw = xo + s * N + j0;
  T* qw = q + s * N + j0;
  const int seg = p.seg;
  const int pb = blockIdx.y * seg;
  const int pe = pb + seg < g.n0 ? pb + seg : g.n0;
  const int a_first = 3 - g.D;  // first differentiated axis

  T zp0[NP];  // z_0 at the previous plane (axis-0 backward neighbour of K^T z), carried along the march
#pragma unroll
  for (int k = 0; k < NP; ++k) zp0[k] = T(0);
  if (PD3O && g.D == 3 && pb - 2 * R0 - 1 >= 0) ldn<T, NP>(zs + (int64_t)(pb - 2 * R0 - 1) * M, zp0);

  // v at plane qp (qp inside [0, n0)), returned by value (a reference into the ring would keep the
  // ring in scratch memory)
  struct VN {
    T v[NP];
  };
  auto load_v = [&](int qp) -> VN {
    VN r;
    T(&v)[NP] = r.v;
    const int64_t off = (int64_t)qp * M;
    if constexpr (!PD3O) {
      ldn<T, NP>(in + off, v);
    } else {
      T u[NP], kt[NP];
      ldn<T, NP>(in + off, u);
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        if (a < a_first) continue;
        const T* zd = zs + (int64_t)(a - a_first) * N + off;
        T zc[NP], zm[NP];
        ldn<T, NP>(zd, zc);
        if (a == 0) {
#pragma unroll
          for (int k = 0; k < NP; ++k) {
            zm[k] = zp0[k];
            zp0[k] = zc[k];
          }
        } else if (a == 1) {
          if (row > 0) {
            ldn<T, NP>(zd - g.n2, zm);
          } else {
#pragma unroll
            for (int k = 0; k < NP; ++k) zm[k] = T(0);
          }
        } else {
          zm[0] = col > 0 ? zd[-1] : T(0);
          if constexpr (NP == 2) zm[1] = zc[0];
        }
        // flipped 2-tap adjoint per direction, summed over directions in order (pxa_gradient2_adjoint)
#pragma unroll
        for (int k = 0; k < NP; ++k) {
          const T term = kt_term<T>(g.c1[a], zm[k], g.c0[a], zc[k]);
          kt[k] = (a == a_first) ? term : kt[k] + term;
        }
      }
      const T one = T(1), mtau = -tau;
#pragma unroll
      for (int k = 0; k < NP; ++k) v[k] = apply_prox<T>(prox, fma(mtau, kt[k], one * u[k]), pw);
      if (qp >= pb && qp < pe) stn<T, NP>(xw + off, v);
    }
    return r;
  };

  if constexpr (R0 == 0) {
    for (int qp = pb; qp < pe; ++qp) (void)load_v(qp);
    return;
  } else {
    T rv[RING][NP], rh[RING][NP];  // v ring and (H0 v) ring, slot = (plane - base) mod RING
#pragma unroll
    for (int r = 0; r < RING; ++r)
#pragma unroll
      for (int k = 0; k < NP; ++k) rv[r][k] = rh[r][k] = T(0);
    const int first = pb - 2 * R0, last = pe - 1 + 2 * R0;
    for (int base = first; base <= last; base += RING) {
      static_for<0, RING>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const int qp = base + j;
        if (qp > last) return;
        if (qp >= 0 && qp < g.n0) {
          const VN r = load_v(qp);
#pragma unroll
          for (int k = 0; k < NP; ++k) rv[j][k] = r.v[k];
        } else {
#pragma unroll
          for (int k = 0; k < NP; ++k) rv[j][k] = T(0);
        }
        // (H0 v)[qp - R0] = sum_t k0[t] v[qp - 2 R0 + t]; zero outside [0, n0) (Trim o S o Pad)
        const int ph = qp - R0;
        constexpr int jh = (j - R0 + RING) % RING;
        if (ph >= 0 && ph < g.n0) {
          T acc[NP];
#pragma unroll
          for (int k = 0; k < NP; ++k) acc[k] = T(0);
          static_for<0, RING>([&](auto TT) {
            constexpr int t = decltype(TT)::value;
            constexpr int slot = (j + 1 + t) % RING;
#pragma unroll
            for (int k = 0; k < NP; ++k) acc[k] = fma(k0[t], rv[slot][k], acc[k]);  // explicit: same bits at every ring position
          });
#pragma unroll
          for (int k = 0; k < NP; ++k) rh[jh][k] = acc[k];
        } else {
#pragma unroll
          for (int k = 0; k < NP; ++k) rh[jh][k] = T(0);
        }
        // Q[i] = (H0^T H0 v)[i] = sum_t k0[t] (H0 v)[i + R0 - t],  i = qp - 2 R0
        const int i = qp - 2 * R0;
        if (i >= pb) {
          T acc[NP];
#pragma unroll
          for (int k = 0; k < NP; ++k) acc[k] = T(0);
          static_for<0, RING>([&](auto TT) {
            constexpr int t = decltype(TT)::value;
            constexpr int slot = ((j - R0 - t) % RING + RING) % RING;
#pragma unroll
            for (int k = 0; k < NP; ++k) acc[k] = fma(k0[t], rh[slot][k], acc[k]);
          });
          stn<T, NP>(qw + (int64_t)i * M, acc);
        }
      });
    }
  }
}

// ------------------------------------------------------------------ kernel B: in-plane G12 + update
template <typename T>
struct PdsB {
  PdsGeom<T> g;
  int tiles1, tiles2;
  unsigned ntiles;
  T k1[2 * kMaxR + 1], k2[2 * kMaxR + 1];
  T g1[kMaxG], g2[kMaxG];
  T tau, rho, omr, pw;
  int prox;
  bool vec_ok;
};

struct PdsPtrs {
  const void* q;    // G0 x (or x when axis 0 is not blurred)
  const void* x;    // x (PD3O: the x written by kernel A)
  const void* u;    // PD3O: u
  const void* z;    // Condat-Vu: z (for K^T z; MODE 2: K^T z itself)
  const void* hty;  // S^T y
  void* w;          // w (input of K in the dual update)
  void* out;        // PD3O: u_new ; Condat-Vu: x_new
};

// MODE: 0 PD3O; 1 Condat-Vu with K^T z gathered from z; 2 Condat-Vu with K^T z precomputed (kernel D)
template <typename T, int R, bool EDGE, int MODE>
__device__ inline void pds_tile(const PdsB<T>& p, const PdsPtrs& P, unsigned char* smem, int64_t img, int ty0,
                                int tx0) {
  using L = Layout<T, R>;
  constexpr int V = L::V;
  constexpr int CA = L::CA;
  constexpr int CW = L::CW;
  T* A = reinterpret_cast<T*>(smem);
  T* PT = A + L::AR * L::AP;
  T* KT = PT + L::AC * L::PTP;
  T* GH = reinterpret_cast<T*>(smem + kGhOff<T, R>);  // boundary-column ghost terms (edge-column tiles)
  const PdsGeom<T>& g = p.g;
  const int n1 = g.n1, n2 = g.n2;
  const int64_t M = (int64_t)n1 * n2;
  const int64_t N = M * g.n0;
  const int64_t s = img / g.n0;
  const int plane = (int)(img - s * g.n0);
  const T* qs = (const T*)P.q + img * M;
  const int tid = threadIdx.x;
  if (EDGE && tid < 2 * R + 1) {
    KT[tid] = p.k1[tid];
    KT[kKT + tid] = p.k2[tid];
  }
  // ---- phase 0: A = Q plane window, zero outside the image
  constexpr int K0 = cdiv(L::N0, kThreads);
#pragma unroll
  for (int k = 0; k < K0; ++k) {
    const int it = tid + k * kThreads;
    if (it < L::N0) {
      const int r = it / L::NGA, c = it - r * L::NGA;
      const int gr = ty0 - 2 * R + r, gc = tx0 - CA + V * c;
      T v[V];
      if (!EDGE) {
        ld_vec<T, V>(qs + (unsigned)(gr * n2 + gc), v);
      } else if (gr >= 0 && gr < n1 && p.vec_ok && gc >= 0 && gc + V <= n2) {
        ld_vec<T, V>(qs + (int64_t)gr * n2 + gc, v);
      } else {
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const bool in = gr >= 0 && gr < n1 && gc + e >= 0 && gc + e < n2;
          v[e] = in ? qs[(int64_t)gr * n2 + gc + e] : T(0);
        }
      }
      st_vec<T, V>(A + r * L::AP + V * c, v);
    }
  }
  __syncthreads();
  // ---- pass A: PT[col][row] = (G1 Q)[row][col]
  constexpr int KA = cdiv(L::NPA, kThreads);
  const bool edge_rows = EDGE && (ty0 < R || ty0 + TY > n1 - R);
#pragma unroll
  for (int k = 0; k < KA; ++k) {
    const int it = tid + k * kThreads;
    if (it < L::NPA) {
      const int a = it % L::NA, b = it / L::NA;
      T acc[V][V];
      sweep<T, R, V, L::AP>(A + (V * a) * L::AP + V * b, p.g1, acc);
      if (edge_rows) ghost_fix<T, R, V, L::AP>(ty0 + V * a, n1, ty0 - 2 * R, A + V * b, p.k1, KT, acc);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        T colv[V];
#pragma unroll
        for (int u = 0; u < V; ++u) colv[u] = acc[u][v];
        st_vec<T, V>(PT + (V * b + v) * L::PTP + V * a, colv);
      }
    }
  }
  __syncthreads();
  // ---- pass B: G2 along rows; results parked in LDS (the PT region, free once every sweep is done)
  constexpr int KB = cdiv(L::NPB, kThreads);
  const bool edge_cols = EDGE && (tx0 < R || tx0 + TX > n2 - R);
  if (edge_cols) {  // the ghost terms of the border columns, by the whole workgroup
    ghost_cols_coop<T, R>(p.k2, PT, GH, tx0, n2);
    __syncthreads();
  }
  using S = Stage<T, R>;
  T st[KB][V][CW];
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    const int it = tid + k * kThreads;
    if (it < L::NPB) {
      int a, cb;
      L::pass_b_item(it, a, cb);
      const int c0 = CW * cb;
      T acc[CW][V];
      sweep<T, R, CW, L::PTP>(PT + (CA - 2 * R + c0) * L::PTP + V * a, p.g2, acc);
      if (edge_cols) ghost_fix_pre<T, R, CW, TY>(tx0 + c0, n2, V * a, GH, KT + kKT, acc);
#pragma unroll
      for (int uu = 0; uu < V; ++uu)
#pragma unroll
        for (int w = 0; w < CW; ++w) st[k][uu][w] = acc[w][uu];
    }
  }
  __syncthreads();  // every G2 sweep is done with PT: O may overwrite it
  T* O = PT;
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    const int it = tid + k * kThreads;
    if (it < L::NPB) {
      int a, cb;
      L::pass_b_item(it, a, cb);
#pragma unroll
      for (int uu = 0; uu < V; ++uu) {
        T* o = O + S::idx(V * a + uu, CW * cb);
#pragma unroll
        for (int w = 0; w < CW; ++w) o[w] = st[k][uu][w];
      }
    }
  }
  __syncthreads();
  // ---- epilogue in row-major order: each V-vector of a tile row is one lane (full 128-B lines for
  // every stream: x, S^T y, u or z, w, out), the solver's point-wise update per element
  const int64_t hoff = ((s % g.y_images) * g.n0 + plane) * M;
  const int a_first = 3 - g.D;
  const T one = T(1), mtau = -p.tau;
  int r0, cq;
  S::lane(tid, r0, cq);
  constexpr int NS = TY / S::RPS;
#pragma unroll
  for (int si = 0; si < NS; ++si) {
    const int r = r0 + si * S::RPS;
    const int gr = ty0 + r, gc = tx0 + V * cq;
    if (EDGE && (gr >= n1 || gc >= n2)) continue;
    const bool full = !EDGE || (p.vec_ok && gc + V <= n2);
    const int64_t off = img * M + (int64_t)gr * n2 + gc;  // voxel offset in x / u / w / out
    const int64_t bo = hoff + (int64_t)gr * n2 + gc;
    auto ld = [&](const void* base, int64_t o, T(&v)[V]) {
      const T* b = (const T*)base + o;
      if (full) {
        ld_vec<T, V>(b, v);
      } else {
#pragma unroll
        for (int e = 0; e < V; ++e) v[e] = gc + e < n2 ? b[e] : T(0);
      }
    };
    auto stv = [&](void* base, int64_t o, const T(&v)[V]) {
      T* b = (T*)base + o;
      if (full) {
        st_vec<T, V>(b, v);
      } else {
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (gc + e < n2) b[e] = v[e];
      }
    };
    T gv[V], xv[V], bv[V], wv[V], ov[V];
    ld_vec<T, V>(O + S::idx(r, V * cq), gv);
    ld(P.x, off, xv);
    ld(P.hty, bo, bv);
    if constexpr (MODE == 0) {
      T uv[V];
      ld(P.u, off, uv);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const T gf = gv[e] - bv[e];                        // grad f(x) = G x - S^T y
        const T ut = one * xv[e] + mtau * gf;              // u_tmp = x - tau grad f(x)
        wv[e] = one * xv[e] + one * ut + (-one) * uv[e];  // x + u_tmp - u
        ov[e] = p.omr * uv[e] + p.rho * ut;               // (1 - rho) u + rho u_tmp
      }
    } else {
      // K^T z at the lane's pixels: sum over directions of c1 z_d[i - e_a] + c0 z_d[i]
      T kt[V];
      if constexpr (MODE == 2) ld(P.z, off, kt);  // written by kernel D (same expression, same bits)
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) {
        if constexpr (MODE == 2) break;
        if (ax < a_first) continue;
        const int64_t zo = (s * g.D + (ax - a_first)) * N + (int64_t)plane * M + (int64_t)gr * n2 + gc;
        T zc[V], zm[V];
        ld(P.z, zo, zc);
        if (ax == 0) {
          if (plane > 0) {
            ld(P.z, zo - M, zm);
          } else {
#pragma unroll
            for (int e = 0; e < V; ++e) zm[e] = T(0);
          }
        } else if (ax == 1) {
          if (gr > 0) {
            ld(P.z, zo - n2, zm);
          } else {
#pragma unroll
            for (int e = 0; e < V; ++e) zm[e] = T(0);
          }
        } else {
          zm[0] = gc > 0 ? ((const T*)P.z)[zo - 1] : T(0);
#pragma unroll
          for (int e = 1; e < V; ++e) zm[e] = zc[e - 1];
        }
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const T term = kt_term<T>(g.c1[ax], zm[e], g.c0[ax], zc[e]);
          kt[e] = (ax == a_first) ? term : kt[e] + term;
        }
      }
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const T gf = gv[e] - bv[e];
        T t = one * xv[e] + mtau * gf;  // x - tau grad f(x)
        t = one * t + mtau * kt[e];     // - tau K^T z
        const T xt = apply_prox<T>(p.prox, t, p.pw);
        wv[e] = T(2) * xt + (-one) * xv[e];   // 2 x_tmp - x
        ov[e] = p.rho * xt + p.omr * xv[e];  // rho x_tmp + (1 - rho) x
      }
    }
    stv(P.w, off, wv);
    stv(P.out, off, ov);
  }
}

template <typename T, int R, int MODE>
__global__ void __launch_bounds__(kThreads, 4) pds_plane_kernel(PdsB<T> p, PdsPtrs P) {
  using L = Layout<T, R>;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const unsigned tile = xcd_tile(blockIdx.x, p.ntiles);
  const unsigned tpi = (unsigned)p.tiles1 * (unsigned)p.tiles2;
  const unsigned img = tile / tpi;
  const unsigned tr = tile - img * tpi;
  const unsigned trow = tr / (unsigned)p.tiles2;
  const int ty0 = (int)trow * TY, tx0 = (int)(tr - trow * (unsigned)p.tiles2) * TX;
  const bool interior = p.vec_ok && (int64_t)p.g.n1 * p.g.n2 <= 0x7fffffff && ty0 - 2 * R >= 0 &&
                        ty0 + TY + 2 * R <= p.g.n1 && tx0 - L::CA >= 0 && tx0 + TX + L::CA <= p.g.n2;
  if (interior)
    pds_tile<T, R, false, MODE>(p, P, smem_raw, img, ty0, tx0);
  else
    pds_tile<T, R, true, MODE>(p, P, smem_raw, img, ty0, tx0);
}

// ------------------------------------------------------------------ host side
template <typename T, int R0, bool PD3O>
int launch_a(const PdsA<T>& pa, int np, int64_t M, int nseg, const void* src, const void* z, void* xo, void* q,
             hipStream_t st) {
  const int64_t blocks = (M + (int64_t)kAThreads * np - 1) / ((int64_t)kAThreads * np);
  dim3 grid((unsigned)blocks, (unsigned)nseg, (unsigned)pa.g.stack);
  if (np == 2)
    hipLaunchKernelGGL((pds_axis0_kernel<T, R0, 2, PD3O>), grid, dim3(kAThreads), 0, st, pa, (const T*)src,
                       (const T*)z, (T*)xo, (T*)q);
  else
    hipLaunchKernelGGL((pds_axis0_kernel<T, R0, 1, PD3O>), grid, dim3(kAThreads), 0, st, pa, (const T*)src,
                       (const T*)z, (T*)xo, (T*)q);
  return last_launch_status();
}

template <typename T, bool PD3O>
int dispatch_a(int R0, const PdsA<T>& pa, int np, int64_t M, int nseg, const void* src, const void* z, void* xo,
               void* q, hipStream_t st) {
  switch (R0) {
    case 0: return launch_a<T, 0, PD3O>(pa, np, M, nseg, src, z, xo, q, st);
    case 1: return launch_a<T, 1, PD3O>(pa, np, M, nseg, src, z, xo, q, st);
    case 2: return launch_a<T, 2, PD3O>(pa, np, M, nseg, src, z, xo, q, st);
    case 3: return launch_a<T, 3, PD3O>(pa, np, M, nseg, src, z, xo, q, st);
    case 4: return launch_a<T, 4, PD3O>(pa, np, M, nseg, src, z, xo, q, st);
    case 5: return launch_a<T, 5, PD3O>(pa, np, M, nseg, src, z, xo, q, st);
    case 6: return launch_a<T, 6, PD3O>(pa, np, M, nseg, src, z, xo, q, st);
    case 7: return launch_a<T, 7, PD3O>(pa, np, M, nseg, src, z, xo, q, st);
    default: return launch_a<T, 8, PD3O>(pa, np, M, nseg, src, z, xo, q, st);
  }
}

template <typename T, int R, int MODE>
int launch_b(const PdsB<T>& pb, const PdsPtrs& P, hipStream_t st) {
  auto kern = pds_plane_kernel<T, R, MODE>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(kGhOff<T, R> + kGhBytes<T, R>));
    attr_set = true;
  }
  const size_t smem = kGhOff<T, R> + kGhBytes<T, R>;  // Layout + the boundary-column ghost terms
  hipLaunchKernelGGL(kern, dim3(pb.ntiles), dim3(kThreads), smem, st, pb, P);
  return last_launch_status();
}

template <typename T, int MODE>
int dispatch_b(int R, const PdsB<T>& pb, const PdsPtrs& P, hipStream_t st) {
  switch (R) {
    case 1: return launch_b<T, 1, MODE>(pb, P, st);
    case 2: return launch_b<T, 2, MODE>(pb, P, st);
    case 3: return launch_b<T, 3, MODE>(pb, P, st);
    case 4: return launch_b<T, 4, MODE>(pb, P, st);
    case 5: return launch_b<T, 5, MODE>(pb, P, st);
    case 6: return launch_b<T, 6, MODE>(pb, P, st);
    case 7: return launch_b<T, 7, MODE>(pb, P, st);
    default: return launch_b<T, 8, MODE>(pb, P, st);
  }
}

int run_a(const PdsA<float>& pa, bool pd3o, int R0, int np, int64_t M, int nseg, const void* src, const void* z,
          void* xo, void* q, hipStream_t st);
int run_a(const PdsA<double>& pa, bool pd3o, int R0, int np, int64_t M, int nseg, const void* src, const void* z,
          void* xo, void* q, hipStream_t st);
int run_b(const PdsB<float>& pb, int mode, int R, const PdsPtrs& P, hipStream_t st);
int run_b(const PdsB<double>& pb, int mode, int R, const PdsPtrs& P, hipStream_t st);

}  // namespace pds
}  // namespace pxa
