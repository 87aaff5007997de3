// Kernel D of the look-ahead PD3O / Condat-Vu step: the dual update of iteration k fused with the
// axis-0 march that opens iteration k + 1 (kernel A's job in the three-launch step of pds3d.hip).
//
// Iteration k ends with z_{k+1} = relax(fenchel_prox_h(z_k + sigma K w_k)) (kernel C); iteration k + 1
// starts with K^T z_{k+1}: PD3O builds v = x_{k+1} = prox_g(u_{k+1} - tau K^T z_{k+1}) and marches G0 v,
// Condat-Vu marches G0 x_{k+1} and kernel B needs K^T z_{k+1}.  Kernel D does both in one pass: at each
// plane of its march a thread updates z at its own positions (stored) and recomputes z_{k+1} at the two
// in-plane backward neighbours K^T z needs (row - 1 for the axis-1 direction, column - 1 for the
// axis-2 one; the axis-0 neighbour is carried from the previous plane), so z_{k+1} is never re-read.
// It writes z_{k+1}, Q = G0 v and (PD3O) x_{k+1} or (Condat-Vu) K^T z_{k+1}.  DUAL = false is the
// first iteration's march (no dual update: z_{k+1} = z).
//
// Compulsory HBM traffic per voxel (fp32, R0 > 0): reads w, z (D fields), u or x; writes z, Q and x or
// K^T z: 40 B at D = 3, against kernel C (28 B) + kernel A (24 B PD3O / 8 B Condat-Vu) in the
// three-launch step.  Requires z_out != z: neighbours read z_k while other threads write z_{k+1}.
#pragma once
#include "pds3d.hpp"

namespace pxa {
namespace pds {

template <typename T>
struct PdsD {
  PdsA<T> a;  // march parameters: geometry, axis-0 taps, tau, prox, segments
  T sigma, lam, rho, omr;
  // soft progress coupling of row neighbours (PXA_TUNE_PDS_MARCH bit 2, A/B; prog == nullptr: off): per unit a
  // counter (launch tag << 16 | planes done) in prog[(s nseg + segment) blocks + blk]; bpr = blocks per row
  unsigned* prog;
  unsigned tag;
  int bpr, lag, nseg, blocks;
};

// Soft coupling (see PdsD): every second plane thread 0 publishes the unit's progress (a vector store), then the
// wavefront reads the row - 1 / row + 1 neighbours' counters through the scalar unit (glc: from the XCD's L2,
// where a same-XCD neighbour's write-through store lands; a vector load would wait for every vector load and
// store in flight, i.e. drain the march: r05z2, 2 x the kernel time even with no waiting) and, while a neighbour
// that has started in this launch (same tag) lags more than `lag` planes behind, sleeps -- at most kCoupleSpins
// times, so that progress never depends on a neighbour being resident.  Only L2 reuse depends on the coupling,
// not correctness.
constexpr int kCoupleSpins = 64;
__device__ __forceinline__ unsigned couple_read(const unsigned* a) {
  unsigned v;
  asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(a) : "memory");
  return v;
}
__device__ __forceinline__ bool couple_lags(unsigned v, unsigned tag, int done, int lag) {
  return (v & 0xFFFF0000u) == tag && (int)(v & 0xFFFFu) + lag < done;
}
__device__ __forceinline__ void couple_step(unsigned* prog, unsigned tag, unsigned me, int64_t up, int64_t dn, int done,
                                            int lag) {
  if (threadIdx.x == 0) __hip_atomic_store(prog + me, tag | (unsigned)done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int spin = 0; spin < kCoupleSpins; ++spin) {
    const bool wait = (up >= 0 && couple_lags(couple_read(prog + up), tag, done, lag)) ||
                      (dn >= 0 && couple_lags(couple_read(prog + dn), tag, done, lag));
    if (!wait) break;
    __builtin_amdgcn_s_sleep(2);
  }
}

// One work unit of kernel D: in-plane block `blk` (kAThreads * NP consecutive positions) of axis-0 segment `segi`
// of volume `s`, marched over the segment's planes (+ the G0 halo planes).
// PF (PXA_TUNE_PDS_MARCH bit 8, DUAL only): every load of plane qp + 1 is issued before plane qp is computed (a
// second register set of the plane's loads, PlaneLoads), so that each wave has two planes of loads in flight; the
// arithmetic is the same expressions on the same values: the same bits.
template <typename T, int NP>
struct PlaneLoads {
  T wf[NP], w1[NP], w2n, zc[3][NP];      // own_z: w at plane + 1, row + 1, the column after the block; z
  T rw[NP], rz[3][NP], rw0[NP], rw2[NP];  // row - 1 neighbours: w, z, w at plane + 1, w at column + 1
  T lw, lz[3], lw0, lw1;                  // column - 1 neighbour: w, z, w at plane + 1, w at row + 1
  T u[NP];                                // u (PD3O) or x (Condat-Vu)
};

template <typename T, int R0, int NP, bool PD3O, bool ISO, bool DUAL, bool NT, bool CP = false, int PF = 0>
__device__ __forceinline__ void march_unit(const PdsD<T>& p, const T* __restrict__ w, const T* __restrict__ z,
                                           const T* __restrict__ src, T* __restrict__ zo, T* __restrict__ ao,
                                           T* __restrict__ q, unsigned blk, int segi, int64_t s) {
  constexpr int RING = 2 * R0 + 1;
  // kernel arguments copied to registers (the lambdas capture by reference; see pds_axis0_kernel)
  const PdsGeom<T> g = p.a.g;
  const T tau = p.a.tau, pw = p.a.pw;
  const int prox = p.a.prox;
  const T sigma = p.sigma, lam = p.lam, rho = p.rho, omr = p.omr;
  T k0[RING];
#pragma unroll
  for (int t = 0; t < RING; ++t) k0[t] = p.a.k0[t];
  const int n0 = g.n0, n1 = g.n1, n2 = g.n2;
  const int64_t M = (int64_t)n1 * n2;
  const int64_t j0 = ((int64_t)blk * kAThreads + threadIdx.x) * NP;
  if (j0 >= M) return;  // no barriers below
  const int64_t N = M * n0;
  const int row = (int)(j0 / n2), col = (int)(j0 - (int64_t)row * n2);
  const T* ws = w + s * N + j0;
  const T* zs = z + s * g.D * N + j0;
  T* zw = zo + s * g.D * N + j0;
  const T* in = src + s * N + j0;
  T* aw = ao + s * N + j0;
  T* qw = q + s * N + j0;
  const int seg = p.a.seg;
  const int pb = segi * seg;
  const int pe = pb + seg < n0 ? pb + seg : n0;
  const int a_first = 3 - g.D;
  const bool row_nb = row + 1 < n1, col_nb = col + NP < n2;

  // z_{k+1} at the thread's own positions of the plane at offset `off`, from w there (wc) and at the next
  // plane (wf)
  auto own_z = [&](int64_t off, const T(&wc)[NP], const T(&wf)[NP], T(&zn)[3][NP]) __attribute__((always_inline)) {
    T w1[NP], w2[NP], zc[3][NP];
    if (row_nb) {
      ldn<T, NP>(ws + off + n2, w1);
    } else {
#pragma unroll
      for (int k = 0; k < NP; ++k) w1[k] = T(0);
    }
#pragma unroll
    for (int k = 0; k + 1 < NP; ++k) w2[k] = wc[k + 1];
    w2[NP - 1] = col_nb ? ws[off + NP] : T(0);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      if (a < a_first) {
#pragma unroll
        for (int k = 0; k < NP; ++k) zc[a][k] = T(0);
      } else {
        ldn<T, NP>(zs + (int64_t)(a - a_first) * N + off, zc[a]);
      }
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      T c3[3], i3[3], n3[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const T wn = a == 0 ? wf[k] : (a == 1 ? w1[k] : w2[k]);
        c3[a] = zc[a][k];
        i3[a] = a < a_first ? T(0) : dual_in<T>(zc[a][k], wc[k], wn, g.c0[a], g.c1[a], sigma);
      }
      dual_out<T, ISO, PD3O>(c3, i3, a_first, lam, rho, omr, n3);
#pragma unroll
      for (int a = 0; a < 3; ++a) zn[a][k] = n3[a];
    }
  };
  // z_{k+1} (all directions) at one position: offset o from the thread's first position, row rr, column
  // cc, plane qp (for aniso TV the unused directions are dead code).  The forward neighbour along
  // direction `back` is the thread's own position, whose w (own_w) is already in a register.
  auto one_z = [&](int64_t o, int qp, int rr, int cc, int back, T own_w, T(&n3)[3]) __attribute__((always_inline)) {
    T c3[3], i3[3];
    const T wc = ws[o];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      if (a < a_first) {
        c3[a] = i3[a] = T(0);
        continue;
      }
      c3[a] = zs[(int64_t)(a - a_first) * N + o];
      T wn;
      if (a == back)
        wn = own_w;
      else if (a == 0)
        wn = qp + 1 < n0 ? ws[o + M] : T(0);
      else if (a == 1)
        wn = rr + 1 < n1 ? ws[o + n2] : T(0);
      else
        wn = cc + 1 < n2 ? ws[o + 1] : T(0);
      i3[a] = dual_in<T>(c3[a], wc, wn, g.c0[a], g.c1[a], sigma);
    }
    dual_out<T, ISO, PD3O>(c3, i3, a_first, lam, rho, omr, n3);
  };

  T wcar[NP];  // DUAL: w at the next plane to process (own positions), carried
  T zp0[NP];   // z_{k+1} of direction 0 at the previous plane (axis-0 backward neighbour of K^T z)
  const int f0 = pb - 2 * R0 > 0 ? pb - 2 * R0 : 0;  // first plane the march visits
#pragma unroll
  for (int k = 0; k < NP; ++k) zp0[k] = wcar[k] = T(0);
  if constexpr (DUAL) {
    ldn<T, NP>(ws + (int64_t)f0 * M, wcar);
    if (g.D == 3 && f0 > 0) {
      T wprev[NP], zt[3][NP];
      ldn<T, NP>(ws + (int64_t)(f0 - 1) * M, wprev);
      own_z((int64_t)(f0 - 1) * M, wprev, wcar, zt);
#pragma unroll
      for (int k = 0; k < NP; ++k) zp0[k] = zt[0][k];
    }
  } else {
    if (g.D == 3 && f0 > 0) ldn<T, NP>(zs + (int64_t)(f0 - 1) * M, zp0);
  }

  struct VN {
    T v[NP];
  };
  // one plane of the march (planes are visited in increasing order from f0): z_{k+1}, K^T z_{k+1}, v
  auto load_v = [&](int qp) __attribute__((always_inline)) -> VN {
    const int64_t off = (int64_t)qp * M;
    const bool mine = qp >= pb && qp < pe;
    T zn[3][NP], zr1[NP], zl2;
    if constexpr (DUAL) {
      T wf[NP];
      if (qp + 1 < n0) {
        ldn<T, NP>(ws + off + M, wf);
      } else {
#pragma unroll
        for (int k = 0; k < NP; ++k) wf[k] = T(0);
      }
      T wc0[NP];
#pragma unroll
      for (int k = 0; k < NP; ++k) wc0[k] = wcar[k];
      own_z(off, wc0, wf, zn);
#pragma unroll
      for (int k = 0; k < NP; ++k) wcar[k] = wf[k];
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        zr1[k] = T(0);
        if (a_first <= 1 && row > 0) {
          T n3[3];
          one_z(off - n2 + k, qp, row - 1, col + k, 1, wc0[k], n3);
          zr1[k] = n3[1];
        }
      }
      zl2 = T(0);
      if (col > 0) {
        T n3[3];
        one_z(off - 1, qp, row, col - 1, 2, wc0[0], n3);
        zl2 = n3[2];
      }
      if (mine) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          if (a < a_first) continue;
          if (NT)
            stn_nt<T, NP>(zw + (int64_t)(a - a_first) * N + off, zn[a]);
          else
            stn<T, NP>(zw + (int64_t)(a - a_first) * N + off, zn[a]);
        }
      }
    } else {
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        if (a < a_first) continue;
        ldn<T, NP>(zs + (int64_t)(a - a_first) * N + off, zn[a]);
      }
#pragma unroll
      for (int k = 0; k < NP; ++k) zr1[k] = T(0);
      if (a_first <= 1 && row > 0) ldn<T, NP>(zs + (int64_t)(1 - a_first) * N + off - n2, zr1);
      zl2 = col > 0 ? zs[(int64_t)(2 - a_first) * N + off - 1] : T(0);
    }
    // K^T z_{k+1}: flipped 2-tap adjoint per direction, summed over directions in order
    // (pxa_gradient2_adjoint; the expression of pds_axis0_kernel and of kernel B's Condat-Vu epilogue)
    T kt[NP];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      if (a < a_first) continue;
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        const T zm = a == 0 ? zp0[k] : (a == 1 ? zr1[k] : (k == 0 ? zl2 : zn[2][k - 1]));
        const T term = kt_term<T>(g.c1[a], zm, g.c0[a], zn[a][k]);
        kt[k] = (a == a_first) ? term : kt[k] + term;
      }
      if (a == 0) {
#pragma unroll
        for (int k = 0; k < NP; ++k) zp0[k] = zn[0][k];
      }
    }
    VN r;
    T(&v)[NP] = r.v;
    if constexpr (PD3O) {
      T u[NP];
      if (NT)
        ldn_nt<T, NP>(in + off, u);
      else
        ldn<T, NP>(in + off, u);
      const T one = T(1), mtau = -tau;
#pragma unroll
      for (int k = 0; k < NP; ++k) v[k] = apply_prox<T>(prox, fma(mtau, kt[k], one * u[k]), pw);
      if (mine) {
        if (NT)
          stn_nt<T, NP>(aw + off, v);
        else
          stn<T, NP>(aw + off, v);
      }
    } else {
      if (NT)
        ldn_nt<T, NP>(in + off, v);
      else
        ldn<T, NP>(in + off, v);
      if (mine) {
        if (NT)
          stn_nt<T, NP>(aw + off, kt);
        else
          stn<T, NP>(aw + off, kt);
      }
    }
    return r;
  };

  // PF: the loads of plane qp (the conditions of own_z / one_z / load_v), then the plane from them
  auto issue = [&](int qp, PlaneLoads<T, NP>& L) __attribute__((always_inline)) {
    const int64_t off = (int64_t)qp * M;
    if (qp + 1 < n0) {
      ldn<T, NP>(ws + off + M, L.wf);
    } else {
#pragma unroll
      for (int k = 0; k < NP; ++k) L.wf[k] = T(0);
    }
    if (row_nb) {
      ldn<T, NP>(ws + off + n2, L.w1);
    } else {
#pragma unroll
      for (int k = 0; k < NP; ++k) L.w1[k] = T(0);
    }
    L.w2n = col_nb ? ws[off + NP] : T(0);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      if (a < a_first) {
#pragma unroll
        for (int k = 0; k < NP; ++k) L.zc[a][k] = T(0);
      } else {
        ldn<T, NP>(zs + (int64_t)(a - a_first) * N + off, L.zc[a]);
      }
    }
    if (a_first <= 1 && row > 0) {
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        const int64_t o = off - n2 + k;
        L.rw[k] = ws[o];
#pragma unroll
        for (int a = 0; a < 3; ++a) L.rz[a][k] = a < a_first ? T(0) : zs[(int64_t)(a - a_first) * N + o];
        L.rw0[k] = qp + 1 < n0 ? ws[o + M] : T(0);
        L.rw2[k] = col + k + 1 < n2 ? ws[o + 1] : T(0);
      }
    }
    if (col > 0) {
      const int64_t o = off - 1;
      L.lw = ws[o];
#pragma unroll
      for (int a = 0; a < 3; ++a) L.lz[a] = a < a_first ? T(0) : zs[(int64_t)(a - a_first) * N + o];
      L.lw0 = qp + 1 < n0 ? ws[o + M] : T(0);
      L.lw1 = row + 1 < n1 ? ws[o + n2] : T(0);
    }
    if (NT)
      ldn_nt<T, NP>(in + off, L.u);
    else
      ldn<T, NP>(in + off, L.u);
  };
  auto compute_v = [&](int qp, const PlaneLoads<T, NP>& L) __attribute__((always_inline)) -> VN {
    const int64_t off = (int64_t)qp * M;
    const bool mine = qp >= pb && qp < pe;
    T zn[3][NP], zr1[NP], zl2;
    T wc0[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) wc0[k] = wcar[k];
    {  // own_z
      T w2[NP];
#pragma unroll
      for (int k = 0; k + 1 < NP; ++k) w2[k] = wc0[k + 1];
      w2[NP - 1] = L.w2n;
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        T c3[3], i3[3], n3[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const T wn = a == 0 ? L.wf[k] : (a == 1 ? L.w1[k] : w2[k]);
          c3[a] = L.zc[a][k];
          i3[a] = a < a_first ? T(0) : dual_in<T>(L.zc[a][k], wc0[k], wn, g.c0[a], g.c1[a], sigma);
        }
        dual_out<T, ISO, PD3O>(c3, i3, a_first, lam, rho, omr, n3);
#pragma unroll
        for (int a = 0; a < 3; ++a) zn[a][k] = n3[a];
      }
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) wcar[k] = L.wf[k];
#pragma unroll
    for (int k = 0; k < NP; ++k) {  // one_z at row - 1 (back = 1: its row + 1 neighbour is the own w)
      zr1[k] = T(0);
      if (a_first <= 1 && row > 0) {
        T c3[3], i3[3], n3[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          if (a < a_first) {
            c3[a] = i3[a] = T(0);
            continue;
          }
          c3[a] = L.rz[a][k];
          const T wn = a == 1 ? wc0[k] : (a == 0 ? L.rw0[k] : L.rw2[k]);
          i3[a] = dual_in<T>(c3[a], L.rw[k], wn, g.c0[a], g.c1[a], sigma);
        }
        dual_out<T, ISO, PD3O>(c3, i3, a_first, lam, rho, omr, n3);
        zr1[k] = n3[1];
      }
    }
    zl2 = T(0);
    if (col > 0) {  // one_z at column - 1 (back = 2)
      T c3[3], i3[3], n3[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        if (a < a_first) {
          c3[a] = i3[a] = T(0);
          continue;
        }
        c3[a] = L.lz[a];
        const T wn = a == 2 ? wc0[0] : (a == 0 ? L.lw0 : L.lw1);
        i3[a] = dual_in<T>(c3[a], L.lw, wn, g.c0[a], g.c1[a], sigma);
      }
      dual_out<T, ISO, PD3O>(c3, i3, a_first, lam, rho, omr, n3);
      zl2 = n3[2];
    }
    if (mine) {
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        if (a < a_first) continue;
        if (NT)
          stn_nt<T, NP>(zw + (int64_t)(a - a_first) * N + off, zn[a]);
        else
          stn<T, NP>(zw + (int64_t)(a - a_first) * N + off, zn[a]);
      }
    }
    T kt[NP];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      if (a < a_first) continue;
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        const T zm = a == 0 ? zp0[k] : (a == 1 ? zr1[k] : (k == 0 ? zl2 : zn[2][k - 1]));
        const T term = kt_term<T>(g.c1[a], zm, g.c0[a], zn[a][k]);
        kt[k] = (a == a_first) ? term : kt[k] + term;
      }
      if (a == 0) {
#pragma unroll
        for (int k = 0; k < NP; ++k) zp0[k] = zn[0][k];
      }
    }
    VN r;
    T(&v)[NP] = r.v;
    if constexpr (PD3O) {
      const T one = T(1), mtau = -tau;
#pragma unroll
      for (int k = 0; k < NP; ++k) v[k] = apply_prox<T>(prox, fma(mtau, kt[k], one * L.u[k]), pw);
      if (mine) {
        if (NT)
          stn_nt<T, NP>(aw + off, v);
        else
          stn<T, NP>(aw + off, v);
      }
    } else {
#pragma unroll
      for (int k = 0; k < NP; ++k) v[k] = L.u[k];
      if (mine) {
        if (NT)
          stn_nt<T, NP>(aw + off, kt);
        else
          stn<T, NP>(aw + off, kt);
      }
    }
    return r;
  };
  (void)issue;
  (void)compute_v;

  if constexpr (R0 == 0) {
    for (int qp = pb; qp < pe; ++qp) (void)load_v(qp);
  } else {
    T rv[RING][NP], rh[RING][NP];
#pragma unroll
    for (int r = 0; r < RING; ++r)
#pragma unroll
      for (int k = 0; k < NP; ++k) rv[r][k] = rh[r][k] = T(0);
    const int first = pb - 2 * R0, last = pe - 1 + 2 * R0;
    // Q = G0 v (the plain two-pass form of pds_axis0_kernel, same taps in the same order) with the two
    // windows held as shift registers: one copy of the plane body.  rv[t] = v at plane qp - 2 R0 + t;
    // rh[t] = (H0 v) at plane qp - 3 R0 + t.  (Static ring slots as in pds_axis0_kernel, i.e. the plane
    // body unrolled RING times, measured no faster: profiles/r03z_pds_march_ring_ab.txt.)
    const bool couple = CP && p.prog != nullptr;  // (CP: a separate instance, so the default keeps its SGPRs)
    PlaneLoads<T, NP> cur, nxt, nx2;
    if constexpr (PF > 0 && DUAL) {
      const int q0 = first < 0 ? 0 : first;
      if (q0 < n0 && q0 <= last) issue(q0, cur);
      if (PF > 1 && q0 + 1 < n0 && q0 + 1 <= last) issue(q0 + 1, nxt);
    }
    const int64_t cbase = (s * p.nseg + segi) * (int64_t)p.blocks;
    const int64_t cup = couple && blk >= (unsigned)p.bpr ? cbase + blk - p.bpr : -1;
    const int64_t cdn = couple && (int64_t)blk + p.bpr < p.blocks ? cbase + blk + p.bpr : -1;
#pragma unroll 1
    for (int qp = first; qp <= last; ++qp) {
      if (couple && ((qp - first) & 1) == 0) couple_step(p.prog, p.tag, (unsigned)(cbase + blk), cup, cdn, qp - first, p.lag);
#pragma unroll
      for (int t = 0; t + 1 < RING; ++t)
#pragma unroll
        for (int k = 0; k < NP; ++k) rv[t][k] = rv[t + 1][k];
      if (qp >= 0 && qp < n0) {
        VN r;
        if constexpr (PF == 1 && DUAL) {
          if (qp + 1 < n0 && qp + 1 <= last) issue(qp + 1, nxt);  // in flight while this plane is computed
          r = compute_v(qp, cur);
          cur = nxt;
        } else if constexpr (PF == 2 && DUAL) {
          if (qp + 2 < n0 && qp + 2 <= last) issue(qp + 2, nx2);  // two planes ahead
          r = compute_v(qp, cur);
          cur = nxt;
          nxt = nx2;
        } else {
          r = load_v(qp);
        }
#pragma unroll
        for (int k = 0; k < NP; ++k) rv[RING - 1][k] = r.v[k];
      } else {
#pragma unroll
        for (int k = 0; k < NP; ++k) rv[RING - 1][k] = T(0);
      }
      // (H0 v)[qp - R0] = sum_t k0[t] v[qp - 2 R0 + t]; zero outside [0, n0) (Trim o S o Pad)
      const int ph = qp - R0;
      T h[NP];
#pragma unroll
      for (int k = 0; k < NP; ++k) h[k] = T(0);
      if (ph >= 0 && ph < n0) {
#pragma unroll
        for (int t = 0; t < RING; ++t)
#pragma unroll
          for (int k = 0; k < NP; ++k) h[k] = fma(k0[t], rv[t][k], h[k]);
      }
#pragma unroll
      for (int t = 0; t + 1 < RING; ++t)
#pragma unroll
        for (int k = 0; k < NP; ++k) rh[t][k] = rh[t + 1][k];
#pragma unroll
      for (int k = 0; k < NP; ++k) rh[RING - 1][k] = h[k];
      // Q[i] = sum_t k0[t] (H0 v)[i + R0 - t],  i = qp - 2 R0
      const int i = qp - 2 * R0;
      if (i >= pb) {
        T acc[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) acc[k] = T(0);
#pragma unroll
        for (int t = 0; t < RING; ++t)
#pragma unroll
          for (int k = 0; k < NP; ++k) acc[k] = fma(k0[t], rh[2 * R0 - t][k], acc[k]);
        if (NT)
          stn_nt<T, NP>(qw + (int64_t)i * M, acc);
        else
          stn<T, NP>(qw + (int64_t)i * M, acc);
      }
    }
  }
}

// Grid over the work units: one workgroup per unit by default; PXA_TUNE_PDS_MARCH bit 1 makes it persistent
// (the resident capacity, a multiple of 8; workgroup w takes units w, w + G, ...).  Units are numbered (volume,
// segment, in-plane block) with the block fastest and the block index XCD-banded (tile2d::xcd_tile), so in the
// persistent form the resident workgroups of an XCD march a contiguous band of rows of one segment, started
// together, and read each other's row - 1 / row + 1 neighbours of w and z from L2.  Measured at 1024^3 (round 5,
// r05c): HBM fetch 25.7 -> 23.8 GiB per launch (1.29 -> 1.19 x compulsory), but kernel D 8.8 -> 11.0 ms (PD3O)
// and 10.2 -> 12.0 ms (Condat-Vu): the marches running in lockstep cost more than the re-fetched rows, so the
// default stays one workgroup per unit, dispatched as slots free up.
template <typename T, int R0, int NP, bool PD3O, bool ISO, bool DUAL, bool NT, bool CP = false, int PF = 0>
__global__ void __launch_bounds__(kAThreads) pds_march_kernel(PdsD<T> p, const T* __restrict__ w,
                                                              const T* __restrict__ z, const T* __restrict__ src,
                                                              T* __restrict__ zo, T* __restrict__ ao,
                                                              T* __restrict__ q, unsigned blocks, unsigned nseg,
                                                              unsigned units) {
  for (unsigned u = blockIdx.x; u < units; u += gridDim.x) {
    const unsigned r = u % blocks, rest = u / blocks;
    march_unit<T, R0, NP, PD3O, ISO, DUAL, NT, CP, PF>(p, w, z, src, zo, ao, q, xcd_tile(r, blocks), (int)(rest % nseg),
                                               (int64_t)(rest / nseg));
  }
}

// ------------------------------------------------------------------ host side
// The coupling's counters: one device buffer per device, grown on demand and zeroed once (tags make old contents
// harmless); launch tags 1..65535 in turn (0 never matches: a zeroed counter reads as "not started").
unsigned* progress_counters(int64_t units);
unsigned next_progress_tag();

template <typename T, int R0, bool PD3O, bool ISO, bool DUAL>
int launch_d(const PdsD<T>& pd, int np, int64_t M, int nseg, const void* w, const void* z, const void* src, void* zo,
             void* ao, void* q, hipStream_t st) {
  // one position per thread by default (occupancy 7 against 4 with two: faster at 1024^3,
  // profiles/r03z_pds_march_ring_ab.txt); PXA_TUNE_PDS_MARCH bit 0 allows two (A/B)
  if (!(tuning(PXA_TUNE_PDS_MARCH) & 1)) np = 1;
  // read-once / write-once streams (src, z_out, x_out or K^T z_out, Q) are non-temporal, so that the re-read
  // neighbour rows of w and z stay in L2 (C3 1024^3, r04b: fetch 29 -> 25.7 B/voxel, PD3O step 15.3 -> 14.4 ms)
  const int64_t blocks = (M + (int64_t)kAThreads * np - 1) / ((int64_t)kAThreads * np);
  const int64_t units = blocks * nseg * pd.a.g.stack;
  PXA_CHECK_ARG(units <= 0x7fffffff);
  // one position per thread: the plane-prefetching march (every load of plane q + 1 issued before plane q is computed;
  // C3 1024^3, r06ao: kernel D 8.78-8.84 -> 8.22-8.23 ms PD3O, 9.74-9.86 -> 8.24-8.25 ms Condat-Vu; same bits).
  // PXA_TUNE_PDS_MARCH bit 8: the march without it, bit 9: two planes ahead (A/B)
  auto kern = np == 2 ? pds_march_kernel<T, R0, 2, PD3O, ISO, DUAL, true> : pds_march_kernel<T, R0, 1, PD3O, ISO, DUAL, true>;
  if constexpr (DUAL) {
    const int64_t tv = tuning(PXA_TUNE_PDS_MARCH);
    if (np == 1 && !(tv & 256))
      kern = (tv & 512) ? pds_march_kernel<T, R0, 1, PD3O, ISO, DUAL, true, false, 2>
                        : pds_march_kernel<T, R0, 1, PD3O, ISO, DUAL, true, false, 1>;
  }
  // grid: one workgroup per unit (PXA_TUNE_PDS_MARCH bit 1: the resident capacity, persistent; see above)
  unsigned grid = (unsigned)units;
  PdsD<T> pdc = pd;
  pdc.prog = nullptr;
  const int64_t bpr = pd.a.g.n2 % ((int64_t)kAThreads * np) == 0 ? pd.a.g.n2 / ((int64_t)kAThreads * np) : 0;
  // (the coupled instance exists for the C3 configuration only: fp32, radius 6, one position per thread)
  constexpr bool kCoupled = std::is_same<T, float>::value && R0 == 6 && DUAL;
  if (kCoupled && (tuning(PXA_TUNE_PDS_MARCH) & 4) && bpr > 0 && np == 1) {
    pdc.prog = progress_counters(units);
    if (pdc.prog == nullptr) return PXA_ERR_ARG;
    pdc.tag = next_progress_tag();
    pdc.bpr = (int)bpr;
    pdc.lag = 2 + (tuning(PXA_TUNE_PDS_MARCH) >> 3);  // planes a neighbour may lag (bits 3+: extra slack)
    pdc.nseg = nseg;
    pdc.blocks = (int)blocks;
  }
  if (tuning(PXA_TUNE_PDS_MARCH) & 2) {
    const unsigned cap = (unsigned)resident_grid((const void*)kern, kAThreads, 0);
    if (grid > cap) grid = cap;
  }
  if constexpr (kCoupled) {
    if (pdc.prog != nullptr) {
      hipLaunchKernelGGL((pds_march_kernel<T, R0, 1, PD3O, ISO, DUAL, true, true>), dim3(grid), dim3(kAThreads), 0, st,
                         pdc, (const T*)w, (const T*)z, (const T*)src, (T*)zo, (T*)ao, (T*)q, (unsigned)blocks,
                         (unsigned)nseg, (unsigned)units);
      return last_launch_status();
    }
  }
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kAThreads), 0, st, pdc, (const T*)w, (const T*)z, (const T*)src, (T*)zo,
                     (T*)ao, (T*)q, (unsigned)blocks, (unsigned)nseg, (unsigned)units);
  return last_launch_status();
}

template <typename T, bool PD3O, bool ISO, bool DUAL>
int dispatch_d(int R0, const PdsD<T>& pd, int np, int64_t M, int nseg, const void* w, const void* z, const void* src,
               void* zo, void* ao, void* q, hipStream_t st) {
  switch (R0) {
    case 0: return launch_d<T, 0, PD3O, ISO, DUAL>(pd, np, M, nseg, w, z, src, zo, ao, q, st);
    case 1: return launch_d<T, 1, PD3O, ISO, DUAL>(pd, np, M, nseg, w, z, src, zo, ao, q, st);
    case 2: return launch_d<T, 2, PD3O, ISO, DUAL>(pd, np, M, nseg, w, z, src, zo, ao, q, st);
    case 3: return launch_d<T, 3, PD3O, ISO, DUAL>(pd, np, M, nseg, w, z, src, zo, ao, q, st);
    case 4: return launch_d<T, 4, PD3O, ISO, DUAL>(pd, np, M, nseg, w, z, src, zo, ao, q, st);
    case 5: return launch_d<T, 5, PD3O, ISO, DUAL>(pd, np, M, nseg, w, z, src, zo, ao, q, st);
    case 6: return launch_d<T, 6, PD3O, ISO, DUAL>(pd, np, M, nseg, w, z, src, zo, ao, q, st);
    case 7: return launch_d<T, 7, PD3O, ISO, DUAL>(pd, np, M, nseg, w, z, src, zo, ao, q, st);
    default: return launch_d<T, 8, PD3O, ISO, DUAL>(pd, np, M, nseg, w, z, src, zo, ao, q, st);
  }
}

// run_d: dual = false is the priming march (ISO irrelevant)
#define PXA_PDS_RUN_D(T)                                                                                         \
  int run_d(const PdsD<T>& pd, bool pd3o, bool iso, bool dual, int R0, int np, int64_t M, int nseg, const void* w, \
            const void* z, const void* src, void* zo, void* ao, void* q, hipStream_t st)
PXA_PDS_RUN_D(float);
PXA_PDS_RUN_D(double);

}  // namespace pds
}  // namespace pxa
