// Dense LinOp (_ExplicitLinOp): Y = X A^T (apply) and Y = X A (adjoint), A row-major (M x N).
//
// HBM-bound for small stacks B (intensity 0.5*B flop/B): stream A exactly once
// with 16 B/lane loads and keep B running sums per lane in registers (B processed in register
// chunks of kBC).  apply: one wavefront per row of A; adjoint: workgroups own (row-chunk x
// column-tile) panels, write partial sums, a second pass adds the chunks in a fixed order.
#include <atomic>
#include "common.hpp"

namespace pxa {
namespace {

constexpr int kBC = 8;  // stacked right-hand sides per register chunk

// 16-B load of A, which every GEMV reads exactly once: non-temporal (streaming) policy, so the matrix
// stream does not evict the re-read vectors (x, 256 KB at N = 65536) from the XCD's 4 MB L2.
template <typename T>
__device__ inline void ld_stream_vec(const T* p, T (&v)[kVecN<T>]) {
  typedef T vt __attribute__((ext_vector_type(kVecN<T>)));
  const vt r = __builtin_nontemporal_load(reinterpret_cast<const vt*>(p));
#pragma unroll
  for (int i = 0; i < kVecN<T>; ++i) v[i] = r[i];
}

// ------------------------------------------------------------------ apply: Y[b, m] = <A[m,:], X[b,:]>
template <typename T>
__global__ void __launch_bounds__(kBlock) gemv_rows_kernel(int64_t M, int64_t N, int64_t B, int64_t b0, int nb,
                                                           const T* __restrict__ A, const T* __restrict__ X,
                                                           T* __restrict__ Y, bool vec) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  constexpr int V = kVecN<T>;
  using VT = typename Vec4<T>::type;
  for (int64_t m = wave; m < M; m += nwaves) {
    const T* a = A + m * N;
    double acc[kBC];
#pragma unroll
    for (int j = 0; j < kBC; ++j) acc[j] = 0.0;
    if (vec) {
      // kU independent 16-B loads of the A row in flight per lane (latency hiding: one wave per row)
      constexpr int kU = 8;
      int64_t k = (int64_t)lane * V;
      for (; k + (kU - 1) * 64 * V < N; k += kU * 64 * V) {
        T av[kU][V];
#pragma unroll
        for (int q = 0; q < kU; ++q) ld_stream_vec<T>(a + k + q * 64 * V, av[q]);  // A read once: streaming policy
#pragma unroll
        for (int q = 0; q < kU; ++q) {
#pragma unroll
          for (int j = 0; j < kBC; ++j) {
            if (j < nb) {
              T xv[V];
              *reinterpret_cast<VT*>(xv) = *reinterpret_cast<const VT*>(X + (b0 + j) * N + k + q * 64 * V);
              T part = T(0);
#pragma unroll
              for (int v = 0; v < V; ++v) part += av[q][v] * xv[v];
              acc[j] += (double)part;
            }
          }
        }
      }
      for (; k < N; k += 64 * V) {
        T av[V];
        ld_stream_vec<T>(a + k, av);
#pragma unroll
        for (int j = 0; j < kBC; ++j) {
          if (j < nb) {
            T xv[V];
            *reinterpret_cast<VT*>(xv) = *reinterpret_cast<const VT*>(X + (b0 + j) * N + k);
            T part = T(0);
#pragma unroll
            for (int v = 0; v < V; ++v) part += av[v] * xv[v];
            acc[j] += (double)part;
          }
        }
      }
    } else {
      for (int64_t k = lane; k < N; k += 64) {
        T av = a[k];
#pragma unroll
        for (int j = 0; j < kBC; ++j)
          if (j < nb) acc[j] += (double)(av * X[(b0 + j) * N + k]);
      }
    }
#pragma unroll
    for (int j = 0; j < kBC; ++j) {
      double v = acc[j];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
      if (lane == 0 && j < nb) Y[(b0 + j) * M + m] = (T)v;
    }
  }
}

// ------------------------------------------------------------------ adjoint: Y[b, n] = sum_m A[m,n] X[b,m]
constexpr int kRowChunk = 128;

template <typename T>
__global__ void __launch_bounds__(kBlock) gemv_cols_partial_kernel(int64_t M, int64_t N, int64_t B, int64_t b0, int nb,
                                                                   const T* __restrict__ A, const T* __restrict__ X,
                                                                   T* __restrict__ part, bool vec) {
  constexpr int V = kVecN<T>;
  const int64_t chunk = blockIdx.y;
  const int64_t m_lo = chunk * kRowChunk;
  const int64_t m_hi = m_lo + kRowChunk < M ? m_lo + kRowChunk : M;
  const int64_t n0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * V;
  if (n0 >= N) return;
  T acc[kBC][V];
#pragma unroll
  for (int j = 0; j < kBC; ++j)
#pragma unroll
    for (int v = 0; v < V; ++v) acc[j][v] = T(0);
#pragma unroll 4
  for (int64_t m = m_lo; m < m_hi; ++m) {
    T av[V];
    if (vec && n0 + V <= N) {
      ld_stream_vec<T>(A + m * N + n0, av);
    } else {
#pragma unroll
      for (int v = 0; v < V; ++v) av[v] = (n0 + v < N) ? A[m * N + n0 + v] : T(0);
    }
#pragma unroll
    for (int j = 0; j < kBC; ++j) {
      if (j < nb) {
        T xm = X[(b0 + j) * M + m];
#pragma unroll
        for (int v = 0; v < V; ++v) acc[j][v] += av[v] * xm;
      }
    }
  }
  // part layout: (chunks, kBC, N)
  T* p = part + chunk * kBC * N;
#pragma unroll
  for (int j = 0; j < kBC; ++j)
    if (j < nb)
#pragma unroll
      for (int v = 0; v < V; ++v)
        if (n0 + v < N) p[j * N + n0 + v] = acc[j][v];
}

template <typename T>
__global__ void __launch_bounds__(kBlock) gemv_cols_final_kernel(int64_t M, int64_t N, int64_t b0, int nb,
                                                                 int64_t chunks, const T* __restrict__ part,
                                                                 T* __restrict__ Y) {
  const int64_t total = (int64_t)nb * N;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    int64_t j = t / N, n = t - j * N;
    double acc = 0.0;
    for (int64_t c = 0; c < chunks; ++c) acc += (double)part[(c * kBC + j) * N + n];
    Y[(b0 + j) * N + n] = (T)acc;
  }
}

// ------------------------------------------------------------------ MFMA path (fp32, B >= kMfmaMinB)
// Y (P x Q) = X (P x K) . op(A),  op(A)[k][q] = A[q][k] (apply: P = B, Q = M, K = N) or A[k][q]
// (adjoint: P = B, Q = N, K = M).  From kMfmaMinB right-hand sides on, A is streamed ONCE through
// v_mfma_f32_32x32x2_f32 (f32 in / f32 accumulate, the exact fmaf chain, 157 TF/s) instead of once per
// kBC-chunk of GEMVs; at B >= ~40 the product turns MFMA-bound.
//
// Fragments (cdna_hip_programming.md §3): lane l supplies Aop[i = l & 31][k-slot h = l >> 5] and
// Bop[k-slot h][j = l & 31]; D[i][j] lands in register r of lane l with j = l & 31,
// i = (r & 3) + 8 (r >> 2) + 4 h.  K advances 16 at a time: MFMA s (0..7) feeds lane half h with
// k = k0 + 8 h + s, so a lane reads 8 CONSECUTIVE k of its X row (two 16-B loads) and, in the apply,
// of its A row (two more); the adjoint's A operand is read along q, coalesced across the 32 lanes.
// A wave owns a (32 PTL) x 32 output block, a 256-thread workgroup four of them along Q (32 PTL x
// 128).  When the P x Q tiles alone cannot fill the chip, K is split over grid.z; the partial slabs
// are summed in a fixed order by a second kernel (deterministic run to run).
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kMfmaMinB = 2;
constexpr int kMfmaQ = 128;  // output columns per workgroup

// Operand fragments of one 16-deep k block (zero outside [0, P) x [kb, ke) x [0, Q)).
template <bool TRANS, int PTL>
__device__ inline void load_block(int64_t k0, int64_t ke, int64_t P, int64_t Q, int64_t K, int64_t p0, int64_t q,
                                  bool qok, int h, int r32, bool vec, const float* __restrict__ X,
                                  const float* __restrict__ A, float (&a)[PTL][8], float (&b)[8]) {
  const int64_t kk = k0 + 8 * h;
  const bool full = vec && kk + 8 <= ke;
#pragma unroll
  for (int t = 0; t < PTL; ++t) {
    const int64_t row = p0 + 32 * t + r32;
    const float* xr = X + row * K + kk;
    if (row < P && full) {
      const float4 lo = *reinterpret_cast<const float4*>(xr);
      const float4 hi = *reinterpret_cast<const float4*>(xr + 4);
      a[t][0] = lo.x; a[t][1] = lo.y; a[t][2] = lo.z; a[t][3] = lo.w;
      a[t][4] = hi.x; a[t][5] = hi.y; a[t][6] = hi.z; a[t][7] = hi.w;
    } else {
#pragma unroll
      for (int s = 0; s < 8; ++s) a[t][s] = (row < P && kk + s < ke) ? xr[s] : 0.f;
    }
  }
  if (!TRANS) {
    const float* ar = A + q * K + kk;
    if (qok && full) {
      const float4 lo = *reinterpret_cast<const float4*>(ar);
      const float4 hi = *reinterpret_cast<const float4*>(ar + 4);
      b[0] = lo.x; b[1] = lo.y; b[2] = lo.z; b[3] = lo.w;
      b[4] = hi.x; b[5] = hi.y; b[6] = hi.z; b[7] = hi.w;
    } else {
#pragma unroll
      for (int s = 0; s < 8; ++s) b[s] = (qok && kk + s < ke) ? ar[s] : 0.f;
    }
  } else {
#pragma unroll
    for (int s = 0; s < 8; ++s) b[s] = (qok && kk + s < ke) ? A[(kk + s) * Q + q] : 0.f;
  }
}

template <int PTL>
__device__ inline void mma_block(const float (&a)[PTL][8], const float (&b)[8], f32x16 (&acc)[PTL]) {
#pragma unroll
  for (int s = 0; s < 8; ++s)
#pragma unroll
    for (int t = 0; t < PTL; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t][s], b[s], acc[t], 0, 0, 0);
}

template <bool TRANS, int PTL>
__global__ void __launch_bounds__(256) mfma_gemm_kernel(int64_t P, int64_t Q, int64_t K, int64_t kchunk,
                                                        const float* __restrict__ X, const float* __restrict__ A,
                                                        float* __restrict__ Y, bool vec) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const int64_t q = (int64_t)blockIdx.x * kMfmaQ + wave * 32 + r32;  // this lane's B / output column
  const int64_t p0 = (int64_t)blockIdx.y * (32 * PTL);
  const int64_t kb = (int64_t)blockIdx.z * kchunk;
  const int64_t ke = kb + kchunk < K ? kb + kchunk : K;
  const bool qok = q < Q;
  f32x16 acc[PTL];
#pragma unroll
  for (int t = 0; t < PTL; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  // two named register buffers: the next block's loads are in flight while this block's MFMAs run
  float a0[PTL][8], b0[8], a1[PTL][8], b1[8];
  load_block<TRANS, PTL>(kb, ke, P, Q, K, p0, q, qok, h, r32, vec, X, A, a0, b0);
  for (int64_t k0 = kb; k0 < ke; k0 += 32) {
    load_block<TRANS, PTL>(k0 + 16, ke, P, Q, K, p0, q, qok, h, r32, vec, X, A, a1, b1);
    mma_block<PTL>(a0, b0, acc);
    if (k0 + 32 < ke) load_block<TRANS, PTL>(k0 + 32, ke, P, Q, K, p0, q, qok, h, r32, vec, X, A, a0, b0);
    if (k0 + 16 < ke) mma_block<PTL>(a1, b1, acc);
  }
  float* Yz = Y + (int64_t)blockIdx.z * P * Q;
  if (qok) {
#pragma unroll
    for (int t = 0; t < PTL; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = p0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < P) Yz[row * Q + q] = acc[t][r];
      }
  }
}

__global__ void __launch_bounds__(kBlock) splitk_sum_kernel(int64_t n, int splits, const float* __restrict__ part,
                                                            float* __restrict__ Y) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float s = part[i];
    for (int z = 1; z < splits; ++z) s += part[(int64_t)z * n + i];  // fixed order
    Y[i] = s;
  }
}

// ---- LDS-staged MFMA GEMM (B >= kLdsMinB, 16-B aligned rows): the MFMA-bound regime of the dense LinOp.
// A 256-thread workgroup owns a (64 BP) x 128 output tile -- all of a B <= 128 stack, so A is streamed from
// HBM exactly once -- as 2 x 2 waves of (32 BP) x 64 (BP x 2 blocks of 32 x 32, one v_mfma_f32_32x32x2_f32
// accumulator each).  K advances by kLdsKt = 32 per stage: the stage's X rows and A rows (apply: A[q][k],
// k contiguous; adjoint: A[k][q], q contiguous) are copied global -> registers -> LDS (double-buffered,
// one barrier per stage; the next stage's global loads are in flight during this stage's MFMAs).  Operand
// fetch follows the fragment map above (lane half h takes k = 8 h + s of a 16-deep block, 8 consecutive k
// per lane = two ds_read_b128 of a [row][k] image, row pitch 36 floats: conflict-free under the
// MI355X_MICROARCH.md §LDS bank model, scripts/ldsbank.py; the adjoint's [k][q] image is read with
// ds_read_b32, 32 consecutive q per lane group).  K is split over the workgroups of a 1-D grid with the
// split index fastest, so that with 8 splits each XCD works on one K slice of X (L2-resident); the partial
// products are summed in a fixed order by splitk_sum_kernel (deterministic run to run).
constexpr int kLdsMinB = 32;
constexpr int kLdsKt = 32;
constexpr int kLdsPitch = kLdsKt + 4;  // [row][k] image pitch (floats)
constexpr int kLdsQPitch = 128 + 4;    // [k][q] image pitch (adjoint's A)

template <bool TRANS, int BP>
struct LdsGemm {
  static constexpr int PT = 64 * BP, QT = 128;
  static constexpr int XS = PT * kLdsPitch;                               // floats per X stage
  static constexpr int AS = TRANS ? kLdsKt * kLdsQPitch : QT * kLdsPitch;  // floats per A stage
  static constexpr int XCH = PT * kLdsKt / 4 / 256;                       // 16-B X chunks per thread per stage
  static constexpr int ACH = QT * kLdsKt / 4 / 256;                       // 16-B A chunks per thread per stage
  static constexpr size_t LDS = (size_t)2 * (XS + AS) * sizeof(float);
};

template <bool TRANS, int BP>
__global__ void __launch_bounds__(256, 2) mfma_lds_kernel(int64_t P, int64_t Q, int64_t K, int64_t kchunk, int splits,
                                                          int gq, const float* __restrict__ X,
                                                          const float* __restrict__ A, float* __restrict__ Y) {
  using G = LdsGemm<TRANS, BP>;
  extern __shared__ __align__(16) float lds[];
  float* Xs = lds;               // [2][PT][kLdsPitch]
  float* As = lds + 2 * G::XS;   // [2][QT][kLdsPitch] or [2][kLdsKt][kLdsQPitch]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const unsigned L = blockIdx.x;
  const int z = (int)(L % (unsigned)splits);
  const unsigned t = L / (unsigned)splits;
  const int64_t q0 = (int64_t)(t % (unsigned)gq) * G::QT;
  const int64_t p0 = (int64_t)(t / (unsigned)gq) * G::PT;
  const int64_t kb = (int64_t)z * kchunk;
  const int64_t ke = kb + kchunk < K ? kb + kchunk : K;
  const int wp0 = (wave >> 1) * 32 * BP, wq0 = (wave & 1) * 64;

  float4 xr[G::XCH], ar[G::ACH];  // one stage in flight, global -> registers
  auto load_stage = [&](int64_t k0) {
#pragma unroll
    for (int u = 0; u < G::XCH; ++u) {
      const int c = tid + 256 * u, row = c >> 3, part = c & 7;
      const int64_t p = p0 + row, k = k0 + 4 * part;
      xr[u] = (p < P && k < ke) ? *reinterpret_cast<const float4*>(X + p * K + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < G::ACH; ++u) {
      const int c = tid + 256 * u;
      if (!TRANS) {
        const int row = c >> 3, part = c & 7;
        const int64_t q = q0 + row, k = k0 + 4 * part;
        ar[u] = (q < Q && k < ke) ? *reinterpret_cast<const float4*>(A + q * K + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        const int kr = c >> 5, part = c & 31;
        const int64_t k = k0 + kr, q = q0 + 4 * part;
        ar[u] = (k < ke && q < Q) ? *reinterpret_cast<const float4*>(A + k * Q + q) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  auto store_stage = [&](int buf) {
    float* xs = Xs + buf * G::XS;
    float* as = As + buf * G::AS;
#pragma unroll
    for (int u = 0; u < G::XCH; ++u) {
      const int c = tid + 256 * u;
      *reinterpret_cast<float4*>(xs + (c >> 3) * kLdsPitch + 4 * (c & 7)) = xr[u];
    }
#pragma unroll
    for (int u = 0; u < G::ACH; ++u) {
      const int c = tid + 256 * u;
      if (!TRANS)
        *reinterpret_cast<float4*>(as + (c >> 3) * kLdsPitch + 4 * (c & 7)) = ar[u];
      else
        *reinterpret_cast<float4*>(as + (c >> 5) * kLdsQPitch + 4 * (c & 31)) = ar[u];
    }
  };

  f32x16 acc[BP][2];
#pragma unroll
  for (int bp = 0; bp < BP; ++bp)
#pragma unroll
    for (int bq = 0; bq < 2; ++bq)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[bp][bq][r] = 0.f;

  load_stage(kb);
  store_stage(0);
  __syncthreads();
  int buf = 0;
  for (int64_t k0 = kb; k0 < ke; k0 += kLdsKt) {
    const bool next = k0 + kLdsKt < ke;
    if (next) load_stage(k0 + kLdsKt);
    const float* xs = Xs + buf * G::XS;
    const float* as = As + buf * G::AS;
#pragma unroll
    for (int k16 = 0; k16 < kLdsKt; k16 += 16) {
      float xf[BP][8], af[2][8];
#pragma unroll
      for (int bp = 0; bp < BP; ++bp) {
        const float* src = xs + (wp0 + 32 * bp + r32) * kLdsPitch + k16 + 8 * h;
        const float4 lo = *reinterpret_cast<const float4*>(src), hi = *reinterpret_cast<const float4*>(src + 4);
        xf[bp][0] = lo.x; xf[bp][1] = lo.y; xf[bp][2] = lo.z; xf[bp][3] = lo.w;
        xf[bp][4] = hi.x; xf[bp][5] = hi.y; xf[bp][6] = hi.z; xf[bp][7] = hi.w;
      }
#pragma unroll
      for (int bq = 0; bq < 2; ++bq) {
        if (!TRANS) {
          const float* src = as + (wq0 + 32 * bq + r32) * kLdsPitch + k16 + 8 * h;
          const float4 lo = *reinterpret_cast<const float4*>(src), hi = *reinterpret_cast<const float4*>(src + 4);
          af[bq][0] = lo.x; af[bq][1] = lo.y; af[bq][2] = lo.z; af[bq][3] = lo.w;
          af[bq][4] = hi.x; af[bq][5] = hi.y; af[bq][6] = hi.z; af[bq][7] = hi.w;
        } else {
#pragma unroll
          for (int s = 0; s < 8; ++s) af[bq][s] = as[(k16 + 8 * h + s) * kLdsQPitch + wq0 + 32 * bq + r32];
        }
      }
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int bp = 0; bp < BP; ++bp)
#pragma unroll
          for (int bq = 0; bq < 2; ++bq)
            acc[bp][bq] = __builtin_amdgcn_mfma_f32_32x32x2f32(xf[bp][s], af[bq][s], acc[bp][bq], 0, 0, 0);
    }
    if (next) store_stage(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  float* Yz = Y + (int64_t)z * P * Q;
#pragma unroll
  for (int bp = 0; bp < BP; ++bp)
#pragma unroll
    for (int bq = 0; bq < 2; ++bq) {
      const int64_t q = q0 + wq0 + 32 * bq + r32;
      if (q >= Q) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = p0 + wp0 + 32 * bp + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < P) Yz[row * Q + q] = acc[bp][bq][r];
      }
    }
}

struct LdsPlan {
  int bp, gq;
  int64_t tiles, splits, kchunk;
};

inline LdsPlan lds_plan(int64_t P, int64_t Q, int64_t K) {
  LdsPlan m;
  m.bp = P > 64 ? 2 : 1;
  const int64_t pt = 64 * m.bp;
  m.gq = (int)((Q + 127) / 128);
  m.tiles = m.gq * ((P + pt - 1) / pt);
  int64_t splits = (512 + m.tiles - 1) / m.tiles;  // two workgroups per CU
  const int64_t max_splits = (K + 511) / 512;      // >= 512 k (16 stages) per slice
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  m.kchunk = ((K + splits - 1) / splits + kLdsKt - 1) / kLdsKt * kLdsKt;
  m.splits = (K + m.kchunk - 1) / m.kchunk;
  return m;
}

// the LDS kernel's operand contract: whole 16-B chunks of rows (X, A) everywhere, at most 128 stacked rows
// per workgroup column
inline bool lds_ok(bool trans, int64_t P, int64_t Q, int64_t K, const float* X, const float* A) {
  return P >= kLdsMinB && P <= 1024 && aligned16(X) && aligned16(A) && K % 4 == 0 && (!trans || Q % 4 == 0);
}

struct MfmaPlan {
  int ptl;
  int64_t gx, gy, splits, kchunk;
};

inline MfmaPlan mfma_plan(int64_t P, int64_t Q, int64_t K) {
  MfmaPlan m;
  m.ptl = P > 32 ? 2 : 1;
  m.gx = (Q + kMfmaQ - 1) / kMfmaQ;
  m.gy = (P + 32 * m.ptl - 1) / (32 * m.ptl);
  const int64_t tiles = m.gx * m.gy;
  int64_t splits = (1024 + tiles - 1) / tiles;  // ~4 workgroups per CU in total
  const int64_t max_splits = (K + 255) / 256;   // keep >= 256 k per slice
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  m.kchunk = ((K + splits - 1) / splits + 15) / 16 * 16;
  m.splits = (K + m.kchunk - 1) / m.kchunk;
  return m;
}

template <bool TRANS, int BP>
int launch_lds(const LdsPlan& m, int64_t P, int64_t Q, int64_t K, const float* X, const float* A, float* out,
               hipStream_t s) {
  using G = LdsGemm<TRANS, BP>;
  auto kern = mfma_lds_kernel<TRANS, BP>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::LDS);
    attr = true;
  }
  const int64_t blocks = m.tiles * m.splits;
  if (blocks > 0x7fffffff) return PXA_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), G::LDS, s, P, Q, K, m.kchunk, (int)m.splits, m.gq, X, A,
                     out);
  return last_launch_status();
}

template <bool TRANS>
int launch_mfma(int64_t P, int64_t Q, int64_t K, const float* X, const float* A, float* Y, float* work,
                hipStream_t s) {
  if (lds_ok(TRANS, P, Q, K, X, A) && tuning(PXA_TUNE_DENSE_KERNEL) == 0) {
    const LdsPlan m = lds_plan(P, Q, K);
    float* out = m.splits > 1 ? work : Y;
    if (m.splits > 1 && work == nullptr) return PXA_ERR_ARG;
    const int e = m.bp == 2 ? launch_lds<TRANS, 2>(m, P, Q, K, X, A, out, s) : launch_lds<TRANS, 1>(m, P, Q, K, X, A, out, s);
    if (e || m.splits == 1) return e;
    hipLaunchKernelGGL(splitk_sum_kernel, dim3(grid_for(P * Q)), dim3(kBlock), 0, s, P * Q, (int)m.splits, work, Y);
    return last_launch_status();
  }
  const MfmaPlan m = mfma_plan(P, Q, K);
  const bool vec = aligned16(X) && (K % 4 == 0) && (TRANS || aligned16(A));
  float* out = m.splits > 1 ? work : Y;
  if (m.splits > 1 && work == nullptr) return PXA_ERR_ARG;
  dim3 grid((unsigned)m.gx, (unsigned)m.gy, (unsigned)m.splits);
  if (m.ptl == 2)
    hipLaunchKernelGGL((mfma_gemm_kernel<TRANS, 2>), grid, dim3(256), 0, s, P, Q, K, m.kchunk, X, A, out, vec);
  else
    hipLaunchKernelGGL((mfma_gemm_kernel<TRANS, 1>), grid, dim3(256), 0, s, P, Q, K, m.kchunk, X, A, out, vec);
  int e = last_launch_status();
  if (e || m.splits == 1) return e;
  hipLaunchKernelGGL(splitk_sum_kernel, dim3(grid_for(P * Q)), dim3(kBlock), 0, s, P * Q, (int)m.splits, work, Y);
  return last_launch_status();
}

inline size_t mfma_workspace_bytes(int64_t P, int64_t Q, int64_t K) {
  const MfmaPlan m = mfma_plan(P, Q, K);
  return m.splits > 1 ? (size_t)m.splits * (size_t)P * (size_t)Q * sizeof(float) : 0;
}


// ------------------------------------------------------------------ normal operator, one pass over A
// Y = s * A^T (A x) + d * x for ONE right-hand side (fp32, N % 4 == 0, N <= kNormMaxN): the
// QuadraticFunc.prox CG operator of ADMM (K^T K + I / tau, opt/solver/pds.py:1645-1653 via
// abc/arithmetic.py ChainRule._quad_spec + AddRule) without the second pass over A.
//
// A 1024-thread workgroup (one per CU: its LDS use excludes a second) owns rows g, g + G, g + 2G, ...
// of A.  A row (N <= 65536 fp32) is held in registers, 16 B per lane-vector, NV vectors per thread
// (64 VGPRs at N = 65536): phase 1 forms t = <A[m,:], x> (x re-read from L2, fp32 4-element partials
// summed in double, fixed-order workgroup reduction), phase 2 adds t * A[m,:] into the workgroup's
// partial of A^T (A x) -- NV - NL vectors per thread in registers, NL in LDS (thread-private slots,
// conflict-free ds_read/write_b128) -- and issues the loads of the next row into each register right
// after its last use, so the next row streams in behind phase 2.  The G partials (G x N fp32) are
// summed in a fixed order by normal_final_kernel: deterministic run to run.  HBM traffic: A once
// (M N 4 B) + 2 G N 4 B of partials (64 MB each way at G = 256, N = 65536) against 2 M N 4 B for
// the apply + adjoint pair.
constexpr int kNormThreads = 1024;
constexpr int kNormMaxN = 65536;
constexpr int kNormG = 256;  // workgroups (fixed: the partition, hence the rounding, does not depend on the device)
constexpr int kNormRegAcc = 7;  // accumulator vectors per thread kept in registers
typedef float nf4 __attribute__((ext_vector_type(4)));

template <int NV>
struct NormPlan {
  static constexpr int NL = NV > kNormRegAcc ? NV - kNormRegAcc : 0;  // accumulator vectors in LDS
  static constexpr int NR = NV - NL;
  static constexpr size_t LDS = (size_t)NL * kNormThreads * 16 + 2 * (kNormThreads / 64) * sizeof(double);
};

// dpp_f64 / wave_sum_f64: common.hpp

// Sum over the 16 doubles the waves of a workgroup left in red[0..15]: lanes 0..15 of every wave read one
// each, a DPP reduction within lane row 0 (fixed order), the total read from lane 0 -- the same bits in
// every wave, one LDS read instead of sixteen in series.
__device__ inline double block_sum16_f64(const double* red, int lane) {
  double v = lane < 16 ? red[lane] : 0.0;
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0x124>(v);
  v += dpp_f64<0x128>(v);
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 0),
                          __builtin_amdgcn_readlane(__double2loint(v), 0));
}

// 16-B buffer loads: the row / x base lives in a scalar resource, the per-vector offset k * 16 KB in a
// scalar offset, the lane offset tid * 16 in ONE vector register shared by every load (global loads would
// hold a 64-bit address per in-flight vector).  Rows are read once (non-temporal, aux 2), x is re-read
// by every row (default policy: it stays in the XCD's L2).
template <int AUX>
__device__ inline float4 buf_ld16(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const nf4 v = __builtin_bit_cast(nf4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, AUX));
  return make_float4(v.x, v.y, v.z, v.w);
}

constexpr int kNormXAhead = 3;  // x vectors loaded ahead of the next row (issued before its loads)

template <int NV, bool FULL>
__global__ void __launch_bounds__(kNormThreads) normal_rows_kernel(int64_t M, int N4, const float* __restrict__ A,
                                                                   const float* __restrict__ x,
                                                                   float* __restrict__ part) {
  using P = NormPlan<NV>;
  constexpr int XA = NV < kNormXAhead ? NV : kNormXAhead;
  extern __shared__ __align__(16) unsigned char nsm[];
  float4* accl = reinterpret_cast<float4*>(nsm);  // [NL][kNormThreads]
  double* red = reinterpret_cast<double*>(nsm + (size_t)P::NL * kNormThreads * 16);  // 2 x 16 (parity)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t G = gridDim.x;
  const int voff = tid * 16;
  const int row_bytes = N4 * 16;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, row_bytes, 0x00020000);
  auto row_rsrc = [&](int64_t r) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(A + r * (int64_t)N4 * 4), (short)0, row_bytes, 0x00020000);
  };
  auto live = [&](int k) { return FULL || tid + k * kNormThreads < N4; };
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 row[NV];
  float4 accr[P::NR];
  float4 xq[XA];
#pragma unroll
  for (int k = 0; k < P::NR; ++k) accr[k] = z4;
#pragma unroll
  for (int k = 0; k < P::NL; ++k) accl[k * kNormThreads + tid] = z4;
  int64_t m = blockIdx.x;
  if (m < M) {
#pragma unroll
    for (int k = 0; k < XA; ++k) xq[k] = live(k) ? buf_ld16<0>(xr, voff, k * kNormThreads * 16) : z4;
    const __amdgpu_buffer_rsrc_t ar = row_rsrc(m);
#pragma unroll
    for (int k = 0; k < NV; ++k) row[k] = live(k) ? buf_ld16<2>(ar, voff, k * kNormThreads * 16) : z4;
  }
  int par = 0;
  for (; m < M; m += G) {
    // phase 1: t = <A[m,:], x>.  The first XA x vectors were loaded before this row (vector loads
    // complete in issue order, so the dot of vector k < XA waits only for row vector k); the rest
    // follow XA ahead of their use.
    double d = 0.0;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const float4 xv = xq[k % XA];
      if (k + XA < NV) xq[k % XA] = live(k + XA) ? buf_ld16<0>(xr, voff, (k + XA) * kNormThreads * 16) : z4;
      float q = row[k].x * xv.x;
      q = fmaf(row[k].y, xv.y, q);
      q = fmaf(row[k].z, xv.z, q);
      q = fmaf(row[k].w, xv.w, q);
      d += (double)q;
    }
    d = wave_sum_f64(d);
    if (lane == 0) red[par * 16 + wave] = d;
    __syncthreads();
    const float t = (float)block_sum16_f64(red + par * 16, lane);
    par ^= 1;  // the next row writes the other half: no second barrier needed
    // phase 2: acc += t * A[m,:]; the next row's first x vectors, then each register refilled with the
    // next row right after its last use (the last row re-reads itself: cache hits, unconditional refills)
    const int64_t mn = m + G;
    const bool more = mn < M;  // uniform
#pragma unroll
    for (int k = 0; k < XA; ++k) xq[k] = live(k) ? buf_ld16<0>(xr, voff, k * kNormThreads * 16) : z4;
    const __amdgpu_buffer_rsrc_t an = row_rsrc(more ? mn : m);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      if (k < P::NR) {
        accr[k].x = fmaf(row[k].x, t, accr[k].x);
        accr[k].y = fmaf(row[k].y, t, accr[k].y);
        accr[k].z = fmaf(row[k].z, t, accr[k].z);
        accr[k].w = fmaf(row[k].w, t, accr[k].w);
      } else {
        float4 a = accl[(k - P::NR) * kNormThreads + tid];
        a.x = fmaf(row[k].x, t, a.x);
        a.y = fmaf(row[k].y, t, a.y);
        a.z = fmaf(row[k].z, t, a.z);
        a.w = fmaf(row[k].w, t, a.w);
        accl[(k - P::NR) * kNormThreads + tid] = a;
      }
      row[k] = live(k) ? buf_ld16<2>(an, voff, k * kNormThreads * 16) : z4;
    }
  }
  float4* out = reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * N4 * 4);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int j = tid + k * kNormThreads;
    if (FULL || j < N4) out[j] = k < P::NR ? accr[k] : accl[(k - P::NR) * kNormThreads + tid];
  }
}

// ---- workgroup groups: each row split in kParts column parts, one per workgroup of a group
// Workgroup (group c, part h) owns the float4 columns [h P4, min((h + 1) P4, N4)) (P4 = ceil(N4 / kParts))
// of rows c, c + C, c + 2C, ... (C = G / kParts groups).  A quarter row is 16 VGPRs per thread at
// N = 65536, so a workgroup holds kBufs = 3 of them -- row i being reduced, rows i + 1 and i + 2 streaming
// in -- plus its part of the A^T (A x) accumulator in registers and its part of x in LDS (64 KB).  Per row:
// the part-dot (per-thread fp32 partials summed in double, DPP wave sum, fixed-order workgroup sum),
// published to the group as two 64-bit words tagged with the launch's tag (relaxed agent-scope stores; each
// word validates itself, no fences), the other parts polled through the scalar unit, t = (float)(((d0 + d1)
// + d2) + d3) in the same order in every member, acc += t * row, the freed buffer refilled with row i + 3.
// While row i is reduced and exchanged, rows i + 1 and i + 2 stream: the one-workgroup-per-row kernel had
// nothing in flight during that time.
// Progress never depends on the other members being resident: a workgroup that waits longer than
// kGroupWaitTicks for a part computes that part-dot itself (the same threads, loads and summation order,
// hence the same bits) and stops waiting for later rows.  Members are g, g ^ 8, g ^ 16, g ^ 24 -- one XCD
// under round-robin dispatch, so the exchange stays in one L2; with fewer than 8 groups (M < 8) every
// workgroup computes all parts itself.  Partials: C x N fp32 (a quarter of the one-workgroup kernel's).
#ifndef PXA_PROBES
#define PXA_PROBES 0
#endif
constexpr bool kGroupProbes = PXA_PROBES != 0;  // probe build: per-workgroup timing stats, store-flavour A/B
constexpr int kParts = 4;
constexpr int kBufs = 4;
constexpr int kGroupWaitTicks = 5000;  // 50 us of the 100 MHz clock
constexpr int kGroupScratch = 2048;    // LDS bytes below the x part

// The CG's p = r' + beta p of the previous step folded into this operator pass (pxa_dense_normal_pdot_pfold): each
// workgroup forms its part of the direction from r' and p (cg_p_kernel's expressions: beta = (float)(||r'||^2 /
// ||r||^2) with ||r'||^2 folded from pxa_cg_update_xr's partials in cg.hip's order, p' = fma(beta, p, r')) instead of
// loading it, group 0's members store p', and workgroup 0 publishes ||r'||^2 as cg_p_kernel does.  Same bits as
// pxa_cg_update followed by pxa_dense_normal_pdot on p'; one launch and one pass over r / p fewer per CG step.
struct PFold {
  const float* r;         // r' (nullptr: no fold, the pass reads x)
  const float* p;         // p of the previous step
  float* pn;              // p' (= the pass's x for the reductions after it)
  const double* rr;       // ||r||^2 of the previous step (device)
  const double* part_rr;  // the ||r'||^2 partials (cg_blocks(n) doubles)
  int nb;
  double* rr_out;         // ||r'||^2 (device): the next step's ||r||^2
  double* rr_host;        // ... into coherent host memory (or nullptr)
  unsigned* flags;        // ... and its completion flag (or nullptr)
  unsigned seq;
};

template <int NVS>
struct GroupPlan {
  static constexpr size_t LDS = (size_t)NVS * kNormThreads * 16 + kGroupScratch;
};

struct GroupGeom {
  int group, part, P4;
};

__device__ inline GroupGeom group_geom(int g, int G, int N4) {
  GroupGeom q;
  if ((G / kParts) % 8 == 0) {
    q.part = (g >> 3) & (kParts - 1);
    q.group = (g >> 5) * 8 + (g & 7);
  } else {
    q.part = g % kParts;
    q.group = g / kParts;
  }
  q.P4 = (N4 + kParts - 1) / kParts;
  return q;
}

// One thread's share of a part-dot: the fp32 fma chain of each of its vectors, summed in double over k
// ascending.  The owner reads the row from registers and x from LDS; a workgroup computing another part's
// dot reads both from memory -- the same values in the same order, hence the same bits.
__device__ inline float dot4(float4 a, float4 b) {
  float q = a.x * b.x;
  q = fmaf(a.y, b.y, q);
  q = fmaf(a.z, b.z, q);
  return fmaf(a.w, b.w, q);
}

// The 8 words of one row's exchange ([part][2]), read through the scalar unit from the XCD's L2 (glc: no
// scalar-cache hit), all requests in flight together.  A vector load would complete only after every vector
// load issued before it -- the rows in flight -- so polling with one would undo the multiple buffering.
__device__ inline void poll_row(const unsigned long long* p, unsigned long long (&w)[8]) {
  asm volatile(
      "s_load_dwordx4 %0, %4, 0x0 glc\n\t"
      "s_load_dwordx4 %1, %4, 0x10 glc\n\t"
      "s_load_dwordx4 %2, %4, 0x20 glc\n\t"
      "s_load_dwordx4 %3, %4, 0x30 glc\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=s"(*reinterpret_cast<__attribute__((ext_vector_type(4))) unsigned*>(&w[0])),
        "=s"(*reinterpret_cast<__attribute__((ext_vector_type(4))) unsigned*>(&w[2])),
        "=s"(*reinterpret_cast<__attribute__((ext_vector_type(4))) unsigned*>(&w[4])),
        "=s"(*reinterpret_cast<__attribute__((ext_vector_type(4))) unsigned*>(&w[6]))
      : "s"(p)
      : "memory");
}

// The lane index, recomputed where it is used: the asm keeps the compiler from hoisting it out of the row
// loop into a register that would then be spilled (a spill reload waits for every load in flight).
__device__ inline int lane_here() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// Workgroup sum of the per-thread doubles d (wave DPP sum, then the fixed-order sum of the 16 wave
// sums); red: 16 doubles of scratch, one barrier.
__device__ inline double group_block_sum(double d, double* red) {
  d = wave_sum_f64(d);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (lane_here() == 0) red[wave] = d;
  __syncthreads();
  return block_sum16_f64(red, lane_here());
}

template <int NVS, bool FULL>
__global__ void __launch_bounds__(kNormThreads) normal_group_kernel(int64_t M, int N4, const float* __restrict__ A,
                                                                    const float* __restrict__ x,
                                                                    float* __restrict__ part,
                                                                    unsigned long long* __restrict__ slots,
                                                                    int rows_per_group, unsigned tag, int solo,
                                                                    unsigned long long* __restrict__ stats, int flav,
                                                                    PFold pf) {
  extern __shared__ __align__(16) unsigned char nsm[];
  // LDS: scratch at the bottom (one base register + immediates): red[b][0, 16) the part-dot sums of buffer
  // b's row, red[3 + b][0, 16) those of a part-dot computed here in another member's place, exch[b][part]
  // the members' part-dots, arrived[b][part] whether they came; then this part of x, [NVS][kNormThreads]
  double* red = reinterpret_cast<double*>(nsm);
  double* exch = red + 6 * 16;
  int* arrived = reinterpret_cast<int*>(exch + kBufs * kParts);
  float4* xs = reinterpret_cast<float4*>(nsm + kGroupScratch);
  const int tid = threadIdx.x;
  const int G = gridDim.x, C = G / kParts;
  const GroupGeom q = group_geom(blockIdx.x, G, N4);
  const int c0 = q.part * q.P4;
  auto width = [&](int h) { return N4 - h * q.P4 < q.P4 ? (N4 - h * q.P4 > 0 ? N4 - h * q.P4 : 0) : q.P4; };
  const int W4 = width(q.part);
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const float4* A4 = reinterpret_cast<const float4*>(A);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  auto live = [&](int k, int w) { return FULL || tid + k * kNormThreads < w; };
  const int voff = tid * 16;
  auto rsrc = [&](const float4* base, int w) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, w * 16, 0x00020000);
  };
  const bool fold = pf.r != nullptr;
  float beta = 0.f;
  if (fold) {
    double rn = 0.0;  // cg.hip fold(): 0 + part[0] + part[1] + ... in order
    for (int j = 0; j < pf.nb; ++j) rn += pf.part_rr[j];
    beta = (float)(rn / pf.rr[0]);
    if (blockIdx.x == 0 && tid == 0) {  // cg_p_kernel's publication of ||r'||^2
      pf.rr_out[0] = rn;
      if (pf.rr_host) pf.rr_host[0] = rn;
      if (pf.flags) {
        __threadfence_system();
        __hip_atomic_store(pf.flags, pf.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  const float4* r4 = reinterpret_cast<const float4*>(pf.r);
  const float4* p4 = reinterpret_cast<const float4*>(pf.p);
  // p' of part h, vector k: fma(beta, p, r') per element (cg_p_kernel's expression)
  auto pfold = [&](int h, int wh, int k) {
    const __amdgpu_buffer_rsrc_t rr_ = rsrc(r4 + h * q.P4, wh), pr_ = rsrc(p4 + h * q.P4, wh);
    const float4 rv = buf_ld16<0>(rr_, voff, k * kNormThreads * 16), pv = buf_ld16<0>(pr_, voff, k * kNormThreads * 16);
    return make_float4(fmaf(beta, pv.x, rv.x), fmaf(beta, pv.y, rv.y), fmaf(beta, pv.z, rv.z), fmaf(beta, pv.w, rv.w));
  };
  if (fold) {
    float4* pn4 = reinterpret_cast<float4*>(pf.pn) + c0;
#pragma unroll
    for (int k = 0; k < NVS; ++k) {
      const float4 v = live(k, W4) ? pfold(q.part, W4, k) : z4;
      xs[k * kNormThreads + tid] = v;
      if (q.group == 0 && live(k, W4)) pn4[tid + k * kNormThreads] = v;
    }
  } else {
    const __amdgpu_buffer_rsrc_t xr = rsrc(x4 + c0, W4);
#pragma unroll
    for (int k = 0; k < NVS; ++k)
      xs[k * kNormThreads + tid] = live(k, W4) ? buf_ld16<0>(xr, voff, k * kNormThreads * 16) : z4;
  }
  const int64_t R = M > q.group ? (M - q.group + C - 1) / C : 0;  // rows of this group
  // four row buffers, four names (no dynamic indexing): when row i is reduced, row i - 1 waits for its
  // members' part-dots and rows i + 1, i + 2 stream in
  float4 b0[NVS], b1[NVS], b2[NVS], b3[NVS];
  float4 acc[NVS];
#pragma unroll
  for (int k = 0; k < NVS; ++k) acc[k] = z4;
  // a part row: unconditional loads (a branch around them would make the compiler's load counting wait for
  // the rows in flight); outside the part the resource's range check returns zeros (the vector offset
  // carries the whole offset, so that the check sees it)
  auto load_row = [&](float4(&bb)[NVS], int64_t r) {
    const __amdgpu_buffer_rsrc_t rr = rsrc(A4 + r * (int64_t)N4 + c0, W4);
#pragma unroll
    for (int k = 0; k < NVS; ++k)
      bb[k] = FULL ? buf_ld16<2>(rr, voff, k * kNormThreads * 16) : buf_ld16<2>(rr, voff + k * kNormThreads * 16, 0);
  };
  // rows are taken as 1 + a multiple of 4 (the loop's shape); padding rows repeat the last row, their t unused
  const int64_t last = q.group + (R > 0 ? R - 1 : 0) * (int64_t)C;
  auto row_of = [&](int64_t i) { const int64_t r = q.group + i * C; return r < last ? r : last; };
  const int64_t Rp = R > 0 ? (R + 2) / 4 * 4 + 1 : 0;  // >= R, = 1 mod 4
  if (R > 0) {
    load_row(b0, row_of(0));
    load_row(b1, row_of(1));
    load_row(b2, row_of(2));
    load_row(b3, row_of(3));
  }
  __syncthreads();  // xs
  // slots: [group][row][part][2 words]
  unsigned long long* gs = slots + (int64_t)q.group * rows_per_group * kParts * 2;
  const unsigned long long want = (unsigned long long)tag << 32;
  // A member's part-dot that does not come in time sets `degraded` (the same in every thread: it is read
  // from LDS after the barrier); from then on the poller looks once per row, the rows still go through the
  // straight-line code below (only the refills as vector loads, so the compiler's load counting stays
  // exact), and the workgroup redoes all its rows without the exchange afterwards.
  int ticks = kGroupWaitTicks;
  bool degraded = false;
  double dm = 0.0;  // this workgroup's part-dot of the row just reduced
  // tid 0: publish row i's part-dot
  auto publish = [&](int64_t i, double v) {
    unsigned long long* rs = gs + i * kParts * 2;
    const unsigned long long hi = (unsigned)__double2hiint(v), lo = (unsigned)__double2loint(v);
    // relaxed agent-scope 8-byte stores (write-through, sc1): the tagged words are visible to the members
    // wherever they run.  Measured (scripts/normal_group_probe.py, r04k): 1.1 us of gather per row against
    // 1.5 us with plain stores, whose line stays in the writer's L2 but reaches the pollers later.
    if (kGroupProbes && (flav & 16)) {  // probe build A/B: plain stores
      __hip_atomic_store(rs + q.part * 2, want | hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_store(rs + q.part * 2 + 1, want | lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
      __hip_atomic_store(rs + q.part * 2, want | hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(rs + q.part * 2 + 1, want | lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  // probe build: tid 0 sums its gather time and poll rounds, tid 64 its time from a step's start to the end
  // of its dot (row arrival) and its barrier wait
  unsigned long long st_gather = 0, st_polls = 0, st_dot = 0, st_bar = 0;
  const unsigned long long st_t0 = kGroupProbes ? (unsigned long long)wall_clock64() : 0;
  // tid 0: the members' part-dots of row i (own = v) into exch[e], arrived[e]
  auto gather = [&](int64_t i, double v, int e) {
    unsigned long long* rs = gs + i * kParts * 2;
    int got = 1 << q.part;
    double w[kParts];
#pragma unroll
    for (int h = 0; h < kParts; ++h) w[h] = v;
    const uint64_t g0 = (uint64_t)wall_clock64();
    const uint64_t until = g0 + (uint64_t)ticks;
    for (;;) {
      unsigned long long pw[8];
      poll_row(rs, pw);
      if (kGroupProbes) ++st_polls;
#pragma unroll
      for (int h = 0; h < kParts; ++h) {
        if (got & (1 << h)) continue;
        const unsigned long long w0 = pw[2 * h], w1 = pw[2 * h + 1];
        if ((w0 >> 32) == tag && (w1 >> 32) == tag) {
          w[h] = __hiloint2double((int)(unsigned)w0, (int)(unsigned)w1);
          got |= 1 << h;
        }
      }
      if (got == (1 << kParts) - 1 || (uint64_t)wall_clock64() > until) break;
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int h = 0; h < kParts; ++h) exch[e * kParts + h] = w[h];
    arrived[e] = got == (1 << kParts) - 1;
    if (kGroupProbes) st_gather += (uint64_t)wall_clock64() - g0;
  };
  // after the barrier: t of the row gathered into exch[e]; acc += t * that row (not for a padding row)
  auto finish = [&](float4(&bb)[NVS], int64_t i, int e) {
    if (!arrived[e]) {
      degraded = true;
      ticks = 0;
    }
    double tot = exch[e * kParts];
#pragma unroll
    for (int h = 1; h < kParts; ++h) tot += exch[e * kParts + h];
    const float t = (float)tot;
    const bool real = i < R;
#pragma unroll
    for (int k = 0; k < NVS; ++k) {
      acc[k].x = real ? fmaf(bb[k].x, t, acc[k].x) : acc[k].x;
      acc[k].y = real ? fmaf(bb[k].y, t, acc[k].y) : acc[k].y;
      acc[k].z = real ? fmaf(bb[k].z, t, acc[k].z) : acc[k].z;
      acc[k].w = real ? fmaf(bb[k].w, t, acc[k].w) : acc[k].w;
    }
    // pin these FMAs before the refill that follows (the asm consumes acc; its memory clobber keeps the
    // loads after it): the buffer's old and new values must not overlap, or the loop-carried buffers get
    // copied at the back edge, and a copy waits for its load
#pragma unroll
    for (int k = 0; k < NVS; ++k) asm volatile("" : "+v"(acc[k].x), "+v"(acc[k].y), "+v"(acc[k].z), "+v"(acc[k].w)::"memory");
  };
  // Row i (buffer cur) is reduced; in the same barrier interval the poller gathers row i - 1's part-dots
  // (published one row earlier, so normally already there); then row i - 1 (buffer prev) is accumulated and
  // prev refilled with row i + 3.  One barrier per row.
  auto step = [&](float4(&cur)[NVS], float4(&prev)[NVS], int64_t i) {
    const uint64_t s0 = kGroupProbes && tid == 64 ? (uint64_t)wall_clock64() : 0;
    double d = 0.0;
#pragma unroll
    for (int k = 0; k < NVS; ++k) d += (double)dot4(cur[k], xs[k * kNormThreads + tid]);
    d = wave_sum_f64(d);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int pi = (int)(i & 1), pe = (int)((i - 1) & 1);
    if (lane_here() == 0) red[pi * 16 + wave] = d;
    uint64_t s1 = 0;
    if (kGroupProbes && tid == 64) {
      s1 = (uint64_t)wall_clock64();
      st_dot += s1 - s0;
    }
    if (tid == 0) gather(i - 1, dm, pe);
    __syncthreads();
    if (kGroupProbes && tid == 64) st_bar += (uint64_t)wall_clock64() - s1;
    dm = block_sum16_f64(red + pi * 16, lane_here());
    if (tid == 0) publish(i, dm);
    finish(prev, i - 1, pe);
    load_row(prev, row_of(i + 3));
  };
  if (!solo && R > 0) {
    {  // row 0
      double d = 0.0;
#pragma unroll
      for (int k = 0; k < NVS; ++k) d += (double)dot4(b0[k], xs[k * kNormThreads + tid]);
      dm = group_block_sum(d, red);
      if (tid == 0) publish(0, dm);
    }
    for (int64_t i = 1; i < Rp; i += 4) {
      step(b1, b0, i);
      step(b2, b1, i + 1);
      step(b3, b2, i + 2);
      step(b0, b3, i + 3);
    }
    // the last row (Rp - 1 = 0 mod 4: buffer b0)
    if (tid == 0) gather(Rp - 1, dm, (int)((Rp - 1) & 1));
    __syncthreads();
    finish(b0, Rp - 1, (int)((Rp - 1) & 1));
  }
  if (solo || degraded) {
    // every row without the exchange: each part-dot computed here from memory -- the same threads, values
    // and summation order as its owner's, hence the same bits as the exchange gives
#pragma unroll
    for (int k = 0; k < NVS; ++k) acc[k] = z4;
    for (int64_t i = 0; i < R; ++i) {
      const int64_t row = q.group + i * C;
      double tot = 0.0;
#pragma unroll 1
      for (int h = 0; h < kParts; ++h) {
        const int wh = width(h);
        const __amdgpu_buffer_rsrc_t ra = rsrc(A4 + row * (int64_t)N4 + h * q.P4, wh);
        const __amdgpu_buffer_rsrc_t rx = rsrc(x4 + h * q.P4, wh);
        double e = 0.0;
#pragma unroll
        for (int k = 0; k < NVS; ++k)
          e += (double)dot4(live(k, wh) ? buf_ld16<2>(ra, voff, k * kNormThreads * 16) : z4,
                            live(k, wh) ? (fold ? pfold(h, wh, k) : buf_ld16<0>(rx, voff, k * kNormThreads * 16)) : z4);
        const double dh = group_block_sum(e, red + (3 + (h & 1)) * 16);  // consecutive sums alternate scratch
        tot = h == 0 ? dh : tot + dh;
      }
      const float t = (float)tot;
      const __amdgpu_buffer_rsrc_t ro = rsrc(A4 + row * (int64_t)N4 + c0, W4);
#pragma unroll
      for (int k = 0; k < NVS; ++k) {
        const float4 a = live(k, W4) ? buf_ld16<2>(ro, voff, k * kNormThreads * 16) : z4;
        acc[k].x = fmaf(a.x, t, acc[k].x);
        acc[k].y = fmaf(a.y, t, acc[k].y);
        acc[k].z = fmaf(a.z, t, acc[k].z);
        acc[k].w = fmaf(a.w, t, acc[k].w);
      }
    }
  }
  if (kGroupProbes) {
    if (tid == 0) {
      stats[blockIdx.x * 8 + 0] = st_t0;
      stats[blockIdx.x * 8 + 1] = (unsigned long long)wall_clock64();
      stats[blockIdx.x * 8 + 2] = st_gather;
      stats[blockIdx.x * 8 + 3] = st_polls;
      stats[blockIdx.x * 8 + 4] = degraded ? 1 : 0;
      stats[blockIdx.x * 8 + 5] = (unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));
    }
    if (tid == 64) {
      stats[blockIdx.x * 8 + 6] = st_dot;
      stats[blockIdx.x * 8 + 7] = st_bar;
    }
  }
  float4* out = reinterpret_cast<float4*>(part) + (int64_t)q.group * N4 + c0;
#pragma unroll
  for (int k = 0; k < NVS; ++k)
    if (live(k, W4)) out[tid + k * kNormThreads] = acc[k];
}

// Fixed-order sum of the G workgroup partials in two launches with enough loads in flight: stage 1
// sums slice y of kNormSlice consecutive partials for one float4 column group per thread (double,
// g ascending); stage 2 adds the G / kNormSlice slice sums (ascending) and forms s * sum + d * x.
constexpr int kNormSlice = 32;

__global__ void __launch_bounds__(kBlock) normal_sum_kernel(int N4, int G, const float4* __restrict__ part,
                                                            double4* __restrict__ sums) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N4) return;
  const int g0 = blockIdx.y * kNormSlice;
  const int g1 = g0 + kNormSlice < G ? g0 + kNormSlice : G;
  double4 acc = make_double4(0.0, 0.0, 0.0, 0.0);
#pragma unroll 8
  for (int g = g0; g < g1; ++g) {
    const float4 v = part[(int64_t)g * N4 + c];
    acc.x += (double)v.x;
    acc.y += (double)v.y;
    acc.z += (double)v.z;
    acc.w += (double)v.w;
  }
  sums[(int64_t)blockIdx.y * N4 + c] = acc;
}

__global__ void __launch_bounds__(kBlock) normal_final_kernel(int N4, int slices, const double4* __restrict__ sums,
                                                              const float4* __restrict__ x, float s, float dd,
                                                              float4* __restrict__ Y) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N4) return;
  double4 acc = sums[c];
  for (int y = 1; y < slices; ++y) {
    const double4 v = sums[(int64_t)y * N4 + c];
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  const float4 xv = x[c];
  Y[c] = make_float4(fmaf(s, (float)acc.x, dd * xv.x), fmaf(s, (float)acc.y, dd * xv.y),
                     fmaf(s, (float)acc.z, dd * xv.z), fmaf(s, (float)acc.w, dd * xv.w));
}

// normal_final + the CG's <p, A p> partials (cg.hip's cg_dot, partition cg_blocks(n)) in one launch, for a
// CG iterating on this operator (after normal_sum, whose slice sums it reads).  Workgroup b owns the cg chunk
// [b chunk, (b + 1) chunk) of the row: its threads form Y as normal_final (slice sums added in slice order)
// for the chunk's float4 columns, keep Y and x in LDS, then form cg_dot's per-thread sums over those copies
// (elements lo + t, lo + t + kBlock, ...) and cg_block_sum.  Same bits as normal_final + cg_dot.
// (A variant that also summed the G partials, normal_sum's 16 MB at C4, ran on only the 64 cg workgroups:
// 11.3 us against 4.6 + 4.5 + 4.5 for the three launches, r05m.)
constexpr int kFdMaxChunk = 2048;  // elements per workgroup (LDS: x and Y, 16 KB)

__global__ void __launch_bounds__(kBlock) normal_final_dot_kernel(int64_t n, int slices, const double4* __restrict__ sums,
                                                                  const float4* __restrict__ x, float s, float dd,
                                                                  float4* __restrict__ Y, int64_t chunk,
                                                                  double* __restrict__ pdot) {
  __shared__ float4 yl[kFdMaxChunk / 4], xl[kFdMaxChunk / 4];
  __shared__ double sh[kBlock / kWave];
  const int64_t N4 = n / 4;
  const int t = threadIdx.x;
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  const int64_t c4lo = lo / 4;
  const int c4n = hi > lo ? (int)((hi - lo) / 4) : 0;
  for (int j = t; j < c4n; j += kBlock) {
    const int64_t c = c4lo + j;
    double4 acc = sums[c];
    for (int y = 1; y < slices; ++y) {
      const double4 v = sums[(int64_t)y * N4 + c];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    const float4 xv = x[c];
    const float4 o = make_float4(fmaf(s, (float)acc.x, dd * xv.x), fmaf(s, (float)acc.y, dd * xv.y),
                                 fmaf(s, (float)acc.z, dd * xv.z), fmaf(s, (float)acc.w, dd * xv.w));
    Y[c] = o;
    yl[j] = o;
    xl[j] = xv;
  }
  __syncthreads();
  const float* yf = reinterpret_cast<const float*>(yl);
  const float* xf = reinterpret_cast<const float*>(xl);
  double acc = 0.0;
  for (int64_t i = t; i < hi - lo; i += kBlock) acc = fma((double)xf[i], (double)yf[i], acc);
  const double r = cg_block_sum(acc, sh);
  if (t == 0) pdot[blockIdx.x] = r;
}

// cg.hip's cg_dot for one fp32 row (the fallback of the fused reduction above)
__global__ void __launch_bounds__(kBlock) normal_pdot_kernel(int64_t n, const float* __restrict__ p,
                                                             const float* __restrict__ ap, double* __restrict__ part) {
  __shared__ double sh[kBlock / kWave];
  const int64_t chunk = (n + gridDim.x - 1) / gridDim.x, lo = blockIdx.x * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  double acc = 0.0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) acc = fma((double)p[i], (double)ap[i], acc);
  const double r = cg_block_sum(acc, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = r;
}

inline int normal_groups(int64_t M) { return (int)(M < kNormG ? M : kNormG); }
// groups of the split kernel: a multiple of 8 (one XCD per group) when M allows, at most kNormG / kParts
inline int normal_group_count(int64_t M) {
  const int64_t cap = kNormG / kParts;
  return (int)(M >= cap ? cap : M >= 8 ? M / 8 * 8 : M);
}
inline int normal_slices(int G) { return (G + kNormSlice - 1) / kNormSlice; }
inline size_t align256(size_t b) { return (b + 255) / 256 * 256; }
inline size_t normal_sums_offset(int G, int64_t N) { return align256((size_t)G * (size_t)N * sizeof(float)); }
// workspace: [partials (<= G x N fp32)][slice sums][pair exchange slots: P x rows per pair x 2 halves x 2 words]
inline size_t normal_slots_offset(int64_t M, int64_t N) {
  const int G = normal_groups(M);
  return normal_sums_offset(G, N) + align256((size_t)normal_slices(G) * (size_t)N * sizeof(double));
}
inline int64_t normal_rows_per_group(int64_t M) {  // padded to 1 + a multiple of 4 (the kernel's row loop)
  const int C = normal_group_count(M);
  return ((M + C - 1) / C + 2) / 4 * 4 + 1;
}
inline size_t normal_stats_offset(int64_t M, int64_t N) {
  return normal_slots_offset(M, N) + align256((size_t)normal_group_count(M) * (size_t)normal_rows_per_group(M) * kParts *
                                              2 * sizeof(uint64_t));
}
// + 64 B per workgroup of probe-build stats
inline size_t normal_workspace(int64_t M, int64_t N) {
  return normal_stats_offset(M, N) + (size_t)kParts * normal_group_count(M) * 8 * sizeof(uint64_t);
}

// fixed-order sum of the `rows` partials (rows x N fp32 at work) and s * sum + d * x; with `pdot`, also the
// CG's <x, Y> partials (cg_blocks(N) doubles, cg.hip's partition and bits)
inline int normal_reduce(int rows, int64_t N, const float* x, float s, float d, float* Y, float* work, double* pdot,
                         hipStream_t st) {
  const int N4 = (int)(N / 4);
  const int slices = normal_slices(rows);
  if (pdot != nullptr) {
    const int nb = cg_blocks(N);
    const int64_t chunk = (N + nb - 1) / nb;
    if (chunk % 4 == 0 && chunk <= kFdMaxChunk) {
      const unsigned cb = (unsigned)((N4 + kBlock - 1) / kBlock);
      double4* sums = reinterpret_cast<double4*>(reinterpret_cast<unsigned char*>(work) + normal_sums_offset(rows, N));
      hipLaunchKernelGGL(normal_sum_kernel, dim3(cb, (unsigned)slices), dim3(kBlock), 0, st, N4, rows,
                         reinterpret_cast<const float4*>(work), sums);
      int e = last_launch_status();
      if (e) return e;
      hipLaunchKernelGGL(normal_final_dot_kernel, dim3(nb), dim3(kBlock), 0, st, N, slices, sums,
                         reinterpret_cast<const float4*>(x), s, d, reinterpret_cast<float4*>(Y), chunk, pdot);
      return last_launch_status();
    }
    const int e = normal_reduce(rows, N, x, s, d, Y, work, nullptr, st);
    if (e) return e;
    hipLaunchKernelGGL(normal_pdot_kernel, dim3(nb), dim3(kBlock), 0, st, N, x, Y, pdot);
    return last_launch_status();
  }
  double4* sums = reinterpret_cast<double4*>(reinterpret_cast<unsigned char*>(work) + normal_sums_offset(rows, N));
  const unsigned cb = (unsigned)((N4 + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(normal_sum_kernel, dim3(cb, (unsigned)slices), dim3(kBlock), 0, st, N4, rows,
                     reinterpret_cast<const float4*>(work), sums);
  int e = last_launch_status();
  if (e) return e;
  hipLaunchKernelGGL(normal_final_kernel, dim3(cb), dim3(kBlock), 0, st, N4, slices, sums,
                     reinterpret_cast<const float4*>(x), s, d, reinterpret_cast<float4*>(Y));
  return last_launch_status();
}

template <int NV>
int launch_normal(int64_t M, int64_t N, const float* A, const float* x, float s, float d, float* Y, float* work,
                  double* pdot, hipStream_t st) {
  using P = NormPlan<NV>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)normal_rows_kernel<NV, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)P::LDS);
    (void)hipFuncSetAttribute((const void*)normal_rows_kernel<NV, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)P::LDS);
    attr = true;
  }
  const int G = normal_groups(M);
  const int N4 = (int)(N / 4);
  if (N4 == NV * kNormThreads)
    hipLaunchKernelGGL((normal_rows_kernel<NV, true>), dim3(G), dim3(kNormThreads), P::LDS, st, M, N4, A, x, work);
  else
    hipLaunchKernelGGL((normal_rows_kernel<NV, false>), dim3(G), dim3(kNormThreads), P::LDS, st, M, N4, A, x, work);
  const int e = last_launch_status();
  return e ? e : normal_reduce(G, N, x, s, d, Y, work, pdot, st);
}

template <int NVS>
int launch_normal_group(int64_t M, int64_t N, const float* A, const float* x, float s, float d, float* Y, float* work,
                        bool solo, double* pdot, hipStream_t st, const PFold& pf = PFold{}) {
  const size_t lds = GroupPlan<NVS>::LDS;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)normal_group_kernel<NVS, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    (void)hipFuncSetAttribute((const void*)normal_group_kernel<NVS, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    attr = true;
  }
  static std::atomic<unsigned> launches{0};
  // exchange tag: a fresh value per launch (slots of earlier launches never match), high byte 0xA5 so that
  // small integers left in a reused workspace do not either
  const unsigned tag = 0xA5000000u | (launches.fetch_add(1) & 0x00FFFFFFu);
  const int C = normal_group_count(M);
  const int N4 = (int)(N / 4);
  const int P4 = (N4 + kParts - 1) / kParts;
  auto* slots = reinterpret_cast<unsigned long long*>(reinterpret_cast<unsigned char*>(work) + normal_slots_offset(M, N));
  const int rpg = (int)normal_rows_per_group(M);
  solo = solo || C % 8 != 0;  // fewer than 8 groups: the members would not share an XCD
  // The tag is baked into the launch arguments: a graph replay would reuse it and accept the previous
  // replay's part-dots from the slots.  Under stream capture every member computes its own parts (solo: no
  // exchange, same bits).
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) solo = true;
  auto* stats = reinterpret_cast<unsigned long long*>(reinterpret_cast<unsigned char*>(work) + normal_stats_offset(M, N));
  const int flav = kGroupProbes ? tuning(PXA_TUNE_NORMAL_KERNEL) : 0;
  if (P4 * kParts == N4 && P4 == NVS * kNormThreads)
    hipLaunchKernelGGL((normal_group_kernel<NVS, true>), dim3(kParts * C), dim3(kNormThreads), lds, st, M, N4, A, x,
                       work, slots, rpg, tag, (int)solo, stats, flav, pf);
  else
    hipLaunchKernelGGL((normal_group_kernel<NVS, false>), dim3(kParts * C), dim3(kNormThreads), lds, st, M, N4, A, x,
                       work, slots, rpg, tag, (int)solo, stats, flav, pf);
  const int e = last_launch_status();
  return e ? e : normal_reduce(C, N, x, s, d, Y, work, pdot, st);
}

}  // namespace
}  // namespace pxa

using namespace pxa;

extern "C" {

size_t pxa_dense_workspace_bytes(int dtype, int trans, int64_t M, int64_t N, int64_t B) {
  if (dtype == PXA_F32 && B >= kMfmaMinB)
    return trans == 0 ? mfma_workspace_bytes(B, M, N) : mfma_workspace_bytes(B, N, M);
  if (trans == 0) return 0;
  size_t es = dtype == PXA_F64 ? 8 : 4;
  int64_t chunks = (M + kRowChunk - 1) / kRowChunk;
  return (size_t)chunks * kBC * (size_t)N * es;
}

int pxa_dense_matmat(int dtype, int trans, int64_t M, int64_t N, int64_t B, const void* A, const void* X, void* Y,
                     void* work, void* stream) {
  PXA_CHECK_ARG(M >= 1 && N >= 1 && B >= 0);
  if (B == 0) return PXA_OK;
  PXA_CHECK_ARG(A != nullptr && X != nullptr && Y != nullptr);
  hipStream_t s = as_stream(stream);
  if (dtype == PXA_F32 && B >= kMfmaMinB) {
    PXA_CHECK_ARG(M * (int64_t)N < ((int64_t)1 << 62));
    if (trans == 0)
      return launch_mfma<false>(B, M, N, (const float*)X, (const float*)A, (float*)Y, (float*)work, s);
    return launch_mfma<true>(B, N, M, (const float*)X, (const float*)A, (float*)Y, (float*)work, s);
  }
  PXA_DISPATCH(dtype, T, {
    bool vec = aligned16(A) && aligned16(X) && (N % kVecN<T> == 0);
    if (trans == 0) {
      int64_t waves = M;
      int grid = grid_for(waves * 64);
      for (int64_t b0 = 0; b0 < B; b0 += kBC) {
        int nb = (int)(B - b0 < kBC ? B - b0 : kBC);
        hipLaunchKernelGGL((gemv_rows_kernel<T>), dim3(grid), dim3(kBlock), 0, s, M, N, B, b0, nb, (const T*)A,
                           (const T*)X, (T*)Y, vec);
        int e = last_launch_status();
        if (e) return e;
      }
      return PXA_OK;
    } else {
      PXA_CHECK_ARG(work != nullptr);
      int64_t chunks = (M + kRowChunk - 1) / kRowChunk;
      PXA_CHECK_ARG(chunks <= 65535);
      int64_t ntiles = (N + (int64_t)kBlock * kVecN<T> - 1) / ((int64_t)kBlock * kVecN<T>);
      bool vecA = aligned16(A) && (N % kVecN<T> == 0);
      for (int64_t b0 = 0; b0 < B; b0 += kBC) {
        int nb = (int)(B - b0 < kBC ? B - b0 : kBC);
        hipLaunchKernelGGL((gemv_cols_partial_kernel<T>), dim3((unsigned)ntiles, (unsigned)chunks), dim3(kBlock), 0, s,
                           M, N, B, b0, nb, (const T*)A, (const T*)X, (T*)work, vecA);
        int e = last_launch_status();
        if (e) return e;
        hipLaunchKernelGGL((gemv_cols_final_kernel<T>), dim3(grid_for((int64_t)nb * N)), dim3(kBlock), 0, s, M, N, b0,
                           nb, chunks, (const T*)work, (T*)Y);
        e = last_launch_status();
        if (e) return e;
      }
      return PXA_OK;
    }
  });
}

size_t pxa_dense_normal_workspace_bytes(int dtype, int64_t M, int64_t N, int64_t B) {
  if (dtype != PXA_F32 || B != 1 || N % 4 != 0 || N > kNormMaxN || M < 1) return 0;
  return normal_workspace(M, N);
}

static int dense_normal(int dtype, int64_t M, int64_t N, int64_t B, const void* A, const void* X, double s, double d, void* Y,
                 void* work, double* pdot, void* stream, const PFold& pf = PFold{}) {
  PXA_CHECK_ARG(M >= 1 && N >= 1 && B >= 0);
  if (B == 0) return PXA_OK;
  PXA_CHECK_ARG(A != nullptr && X != nullptr && Y != nullptr && Y != X);
  if (dtype != PXA_F32 && dtype != PXA_F64) return PXA_ERR_DTYPE;
  if (pxa_dense_normal_workspace_bytes(dtype, M, N, B) == 0) return PXA_ERR_UNSUPPORTED;
  PXA_CHECK_ARG(work != nullptr && aligned16(A) && aligned16(X) && aligned16(Y) && aligned16(work));
  hipStream_t st = as_stream(stream);
  const float* a = (const float*)A;
  const float* x = (const float*)X;
  const float fs = (float)s, fd = (float)d;
  float* y = (float*)Y;
  float* w = (float*)work;
  const int kern = tuning(PXA_TUNE_NORMAL_KERNEL) & 15;  // (probe build: bit 4 selects plain exchange stores)
  if (kern != 1) {  // split rows (2: without the exchange, every part-dot computed by every member; same bits)
    const int64_t nvs = ((N / 4 + kParts - 1) / kParts + kNormThreads - 1) / kNormThreads;  // vectors per part
    const bool solo = kern == 2;
    if (nvs <= 1) return launch_normal_group<1>(M, N, a, x, fs, fd, y, w, solo, pdot, st, pf);
    if (nvs <= 2) return launch_normal_group<2>(M, N, a, x, fs, fd, y, w, solo, pdot, st, pf);
    return launch_normal_group<4>(M, N, a, x, fs, fd, y, w, solo, pdot, st, pf);
  }
  if (pf.r != nullptr) return PXA_ERR_UNSUPPORTED;  // (the one-workgroup-per-row A/B kernel has no fold)
  const int64_t nv = (N / 4 + kNormThreads - 1) / kNormThreads;  // vectors per thread
  if (nv <= 1) return launch_normal<1>(M, N, a, x, fs, fd, y, w, pdot, st);
  if (nv <= 2) return launch_normal<2>(M, N, a, x, fs, fd, y, w, pdot, st);
  if (nv <= 4) return launch_normal<4>(M, N, a, x, fs, fd, y, w, pdot, st);
  if (nv <= 8) return launch_normal<8>(M, N, a, x, fs, fd, y, w, pdot, st);
  if (nv <= 12) return launch_normal<12>(M, N, a, x, fs, fd, y, w, pdot, st);
  return launch_normal<16>(M, N, a, x, fs, fd, y, w, pdot, st);
}

int pxa_dense_normal(int dtype, int64_t M, int64_t N, int64_t B, const void* A, const void* X, double s, double d,
                     void* Y, void* work, void* stream) {
  return dense_normal(dtype, M, N, B, A, X, s, d, Y, work, nullptr, stream);
}

int pxa_dense_normal_pdot(int dtype, int64_t M, int64_t N, const void* A, const void* X, double s, double d, void* Y,
                          void* work, double* pdot, void* stream) {
  PXA_CHECK_ARG(pdot != nullptr);
  return dense_normal(dtype, M, N, 1, A, X, s, d, Y, work, pdot, stream);
}

int pxa_dense_normal_pdot_pfold(int dtype, int64_t M, int64_t N, const void* A, const void* R, const void* P, void* P_new,
                                const double* rr, const double* part_rr, double* rr_out, double* rr_host, uint32_t* flags,
                                uint32_t seq, double s, double d, void* Y, void* work, double* pdot, void* stream) {
  PXA_CHECK_ARG(pdot != nullptr && R != nullptr && P != nullptr && P_new != nullptr && rr != nullptr && part_rr != nullptr &&
                rr_out != nullptr);
  PXA_CHECK_ARG(P_new != P && P_new != R && P_new != Y && aligned16(R) && aligned16(P) && aligned16(P_new));
  PXA_CHECK_ARG(dtype == PXA_F32 && rr_out != rr);
  PFold pf;
  pf.r = (const float*)R;
  pf.p = (const float*)P;
  pf.pn = (float*)P_new;
  pf.rr = rr;
  pf.part_rr = part_rr;
  pf.nb = cg_blocks(N);
  pf.rr_out = rr_out;
  pf.rr_host = rr_host;
  pf.flags = (unsigned*)flags;
  pf.seq = (unsigned)seq;
  // X = p': the reductions after the pass read it (d p', <p', A p'>); the pass itself forms its parts from r' and p
  return dense_normal(dtype, M, N, 1, A, P_new, s, d, Y, work, pdot, stream, pf);
}

}  // extern "C"
