// Element-wise kernels: operator-algebra glue, solver updates and the separable proxes.
//
// HBM-bound streaming: 16 B per lane per access (float4 / double2), grid-stride over at most
// 8 workgroups per CU.  A scalar tail handles n % V and unaligned views.
#include "common.hpp"

namespace pxa {
namespace {

// ---------------------------------------------------------------- generic vectorised map
// Op::operator()(T* v[NIN], T& out) style is awkward in device code; use per-element functors
// that receive the element index so each kernel reads exactly what it needs.
template <typename T, int NIN, typename Op>
// `out` may alias an input (solver updates written in place): element i is read and written by the
// same thread only, so no __restrict__ on the operands.
__global__ void __launch_bounds__(kBlock) map_kernel(int64_t n, Op op, const T* a, const T* b, const T* c, T* out,
                                                     bool vec) {
  constexpr int V = kVecN<T>;
  using VT = typename Vec4<T>::type;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t nv = vec ? n / V : 0;
  for (int64_t i = tid; i < nv; i += stride) {
    T va[V], vb[V], vc[V], vo[V];
    *reinterpret_cast<VT*>(va) = reinterpret_cast<const VT*>(a)[i];
    if (NIN > 1) *reinterpret_cast<VT*>(vb) = reinterpret_cast<const VT*>(b)[i];
    if (NIN > 2) *reinterpret_cast<VT*>(vc) = reinterpret_cast<const VT*>(c)[i];
#pragma unroll
    for (int k = 0; k < V; ++k) vo[k] = op(va[k], NIN > 1 ? vb[k] : T(0), NIN > 2 ? vc[k] : T(0));
    reinterpret_cast<VT*>(out)[i] = *reinterpret_cast<VT*>(vo);
  }
  for (int64_t i = nv * V + tid; i < n; i += stride) {
    out[i] = op(a[i], NIN > 1 ? b[i] : T(0), NIN > 2 ? c[i] : T(0));
  }
}

template <typename T, int NIN, typename Op>
int launch_map(int64_t n, Op op, const void* a, const void* b, const void* c, void* out, void* stream) {
  PXA_CHECK_ARG(n >= 0);
  if (n == 0) return PXA_OK;
  PXA_CHECK_ARG(a != nullptr && out != nullptr);
  if (NIN > 1) PXA_CHECK_ARG(b != nullptr);
  if (NIN > 2) PXA_CHECK_ARG(c != nullptr);
  bool vec = aligned16(a) && aligned16(out) && (NIN < 2 || aligned16(b)) && (NIN < 3 || aligned16(c));
  int64_t items = vec ? (n + kVecN<T> - 1) / kVecN<T> : n;
  hipLaunchKernelGGL((map_kernel<T, NIN, Op>), dim3(grid_for(items)), dim3(kBlock), 0, as_stream(stream), n, op,
                     (const T*)a, (const T*)b, (const T*)c, (T*)out, vec);
  return last_launch_status();
}

// The contractions of a*x + b*y (+ c*z) are spelled out: with -ffp-contract=fast the backend picks which
// product to fuse per kernel, and a fused kernel reusing these functors (admm_l1_kernel, the PDS marches'
// fma(b, y, a * x)) must round exactly like the map launches it replaces.
template <typename T>
struct AxpbyOp {
  T a, b;
  __device__ T operator()(T x, T y, T) const { return fma(b, y, a * x); }
};
template <typename T>
struct ScaleOp {
  T a;
  __device__ T operator()(T x, T, T) const { return a * x; }
};
template <typename T>
struct ExtrapOp {  // (x - y) * a + x   (PGD momentum, pgd.py:179-181)
  T a;
  __device__ T operator()(T x, T y, T) const {
    T d = x - y;
    d = d * a;
    return d + x;
  }
};
template <typename T>
struct Lin3Op {
  T a, b, c;
  __device__ T operator()(T x, T y, T z) const { return fma(c, z, fma(b, y, a * x)); }
};
template <typename T>
struct DivOp {
  T d;
  __device__ T operator()(T x, T, T) const { return x / d; }
};
template <typename T>
struct AddScalarOp {
  T s;
  __device__ T operator()(T x, T, T) const { return x + s; }
};
template <typename T>
struct FillOp {
  T v;
  __device__ T operator()(T, T, T) const { return v; }
};
template <typename T>
struct MulOp {
  __device__ T operator()(T x, T y, T) const { return x * y; }
};
template <typename T>
struct ClipOp {
  T lo, hi;
  bool has_hi;
  __device__ T operator()(T x, T, T) const {
    // numpy clip(x, lo, None): max(x, lo); NaN propagates like numpy.
    T r = x < lo ? lo : x;
    if (has_hi) r = r > hi ? hi : r;
    return r;
  }
};

// L1Norm.prox: fmax(0, |x| - tau) * sign(x)   (norm.py:47-52)
template <typename T>
__device__ inline T soft(T x, T tau) {
  T m = fabs(x) - tau;
  m = m > T(0) ? m : T(0);
  T s = x > T(0) ? T(1) : (x < T(0) ? T(-1) : T(0));
  return m * s;
}

template <typename T>
struct ProxL1Op {
  T tau;
  __device__ T operator()(T x, T, T) const { return soft(x, tau); }
};
// x - sigma * prox_{lam/sigma}(x / sigma)
template <typename T>
struct FenchelL1Op {
  T sigma, t;  // t = (1/sigma) * lam, computed in T on the host exactly like the reference
  __device__ T operator()(T x, T, T) const {
    T p = soft(x / sigma, t);
    return p * (-sigma) + x;
  }
};
// scale * (x - prox_{mu}(x)) / mu
template <typename T>
struct MoreauL1Op {
  T mu, scale;
  __device__ T operator()(T x, T, T) const {
    T r = x - soft(x, mu);
    r = r / mu;
    return r * scale;
  }
};

// ---------------------------------------------------------------- grouped (L21) kernels
// x viewed as (outer, group, inner): one thread per (outer, inner) column.
enum GroupMode { kProx = 0, kFenchel = 1, kMoreau = 2, kNorm = 3 };

template <typename T, int MODE>
__global__ void __launch_bounds__(kBlock) group_kernel(int64_t outer, int64_t group, int64_t inner,
                                                       const T* x, T* out, T p0, T p1, T p2) {  // out may alias x
  const int64_t total = outer * inner;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    int64_t o = t / inner, i = t - o * inner;
    const T* xp = x + o * group * inner + i;
    T* op = out + o * group * inner + i;
    // Pass 1: l2 norm over the group (reference: (arr**2).sum(l2_axis); sqrt).
    T s = T(0);
    for (int64_t g = 0; g < group; ++g) {
      T v = xp[g * inner];
      if (MODE == kFenchel) v = v / p0;
      s += v * v;
    }
    T n = sqrt(s);
    if (MODE == kNorm) {
      out[t] = n;
      continue;
    }
    T tau = (MODE == kProx) ? p0 : (MODE == kFenchel ? p1 : p0);
    T f = T(1) - tau / (n > tau ? n : tau);  // 1 - tau / fmax(n, tau)
    for (int64_t g = 0; g < group; ++g) {
      T v = xp[g * inner];
      T r;
      if (MODE == kProx) {
        r = v * f;
      } else if (MODE == kFenchel) {  // x - sigma * prox(x/sigma, lam/sigma)
        T p = (v / p0) * f;
        r = p * (-p0) + v;
      } else {  // kMoreau: scale * (x - prox_mu(x)) / mu
        r = (v - v * f) / p0;
        r = r * p2;
      }
      op[g * inner] = r;
    }
  }
}

// The same arithmetic for G = 2 / 3 (the Gradient's directions: L21 over D fields), 16-B vectors along
// inner, outer on grid.y: a thread reads its G vectors once (the scalar kernel above reads every value
// twice, 4 B per lane, behind a 64-bit division per element: 0.37 of HBM at 1024^3) and two column blocks
// per iteration are in flight.
template <typename T, int MODE, int G>
__device__ inline void group_vec_one(const T (&v)[G][kVecN<T>], T (&r)[G][kVecN<T>], T (&nv)[kVecN<T>], T p0, T p1,
                                     T p2) {
#pragma unroll
  for (int e = 0; e < kVecN<T>; ++e) {
    T s = T(0);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      T w = v[g][e];
      if (MODE == kFenchel) w = w / p0;
      s += w * w;
    }
    const T n = sqrt(s);
    nv[e] = n;
    const T tau = (MODE == kProx) ? p0 : (MODE == kFenchel ? p1 : p0);
    const T f = T(1) - tau / (n > tau ? n : tau);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const T w = v[g][e];
      T q;
      if (MODE == kProx) {
        q = w * f;
      } else if (MODE == kFenchel) {
        const T pr = (w / p0) * f;
        q = pr * (-p0) + w;
      } else {
        q = (w - w * f) / p0;
        q = q * p2;
      }
      r[g][e] = q;
    }
  }
}

template <typename T, int MODE, int G>
__global__ void __launch_bounds__(kBlock) group_vec_kernel(int64_t inner_v, int64_t inner, const T* x, T* out, T p0,
                                                           T p1, T p2) {  // out may alias x
  constexpr int V = kVecN<T>;
  using VT = typename Vec4<T>::type;
  const int64_t o = blockIdx.y;
  const VT* xo = reinterpret_cast<const VT*>(x + o * G * inner);
  VT* oo = reinterpret_cast<VT*>(out + (MODE == kNorm ? o * inner : o * G * inner));
  const int64_t iv = inner / V;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // read once, written once: non-temporal both ways
  typedef T nvt __attribute__((ext_vector_type(V)));
  const nvt* xn = reinterpret_cast<const nvt*>(xo);
  nvt* on = reinterpret_cast<nvt*>(oo);
  auto put = [&](int64_t t, const T (&r)[G][V], const T (&nv)[V]) {
    if (MODE == kNorm) {
      __builtin_nontemporal_store(*reinterpret_cast<const nvt*>(nv), on + t);
    } else {
#pragma unroll
      for (int g = 0; g < G; ++g) __builtin_nontemporal_store(*reinterpret_cast<const nvt*>(r[g]), on + g * iv + t);
    }
  };
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < inner_v; t += 2 * stride) {
    const int64_t t2 = t + stride;
    const bool two = t2 < inner_v;
    T a[G][V], b[G][V], r[G][V], nv[V];
#pragma unroll
    for (int g = 0; g < G; ++g) *reinterpret_cast<nvt*>(a[g]) = __builtin_nontemporal_load(xn + g * iv + t);
    if (two) {
#pragma unroll
      for (int g = 0; g < G; ++g) *reinterpret_cast<nvt*>(b[g]) = __builtin_nontemporal_load(xn + g * iv + t2);
    }
    group_vec_one<T, MODE, G>(a, r, nv, p0, p1, p2);
    put(t, r, nv);
    if (two) {
      group_vec_one<T, MODE, G>(b, r, nv, p0, p1, p2);
      put(t2, r, nv);
    }
  }
}

template <typename T, int MODE>
int launch_group(int64_t outer, int64_t group, int64_t inner, const void* x, void* out, double p0, double p1,
                 double p2, void* stream) {
  PXA_CHECK_ARG(outer >= 0 && group >= 1 && inner >= 0);
  if (outer * inner == 0) return PXA_OK;
  PXA_CHECK_ARG(x != nullptr && out != nullptr);
  constexpr int V = kVecN<T>;
  if ((group == 2 || group == 3) && inner % V == 0 && outer <= 65535 && aligned16(x) && aligned16(out)) {
    const int64_t inner_v = inner / V;
    const int64_t want = (inner_v + 2 * kBlock - 1) / (2 * kBlock);
    const int gx = (int)(want < (int64_t)kMaxGrid ? want : (int64_t)kMaxGrid);
    const dim3 grid((unsigned)(gx > 0 ? gx : 1), (unsigned)outer);
    if (group == 2)
      hipLaunchKernelGGL((group_vec_kernel<T, MODE, 2>), grid, dim3(kBlock), 0, as_stream(stream), inner_v, inner,
                         (const T*)x, (T*)out, (T)p0, (T)p1, (T)p2);
    else
      hipLaunchKernelGGL((group_vec_kernel<T, MODE, 3>), grid, dim3(kBlock), 0, as_stream(stream), inner_v, inner,
                         (const T*)x, (T*)out, (T)p0, (T)p1, (T)p2);
    return last_launch_status();
  }
  hipLaunchKernelGGL((group_kernel<T, MODE>), dim3(grid_for(outer * inner)), dim3(kBlock), 0, as_stream(stream),
                     outer, group, inner, (const T*)x, (T*)out, (T)p0, (T)p1, (T)p2);
  return last_launch_status();
}

// out[i] = a*x[i] + b*y[i % ny]   (stack broadcast of a (ny,) vector; ArgShiftRule / AddRule)
template <typename T>
__global__ void __launch_bounds__(kBlock) bcast_kernel(int64_t n, int64_t ny, T a, const T* x, T b,
                                                       const T* __restrict__ y, T* out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = a * x[i] + b * y[i % ny];
}

// out[r, i] = y[r, i] + s * c[r] * x[r, i]   (per-row step of CG on stacked right-hand sides, cg.py:125-153)
// out may alias x or y (CG: x += a p, r -= a A p, p = r + b p): no __restrict__ on those three; each
// element is read and written by the same thread only.
template <typename T>
__global__ void __launch_bounds__(kBlock) axpy_rows_kernel(int64_t rows, int64_t n, const T* __restrict__ c, T s,
                                                           const T* x, const T* y, T* out) {
  const int64_t total = rows * n;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const T a = s * c[i / n];
    out[i] = a * x[i] + y[i];
  }
}

// out[r] = (T)(num[r] / den[r]) in float64 (CG alpha = ||r||^2 / <p, A p>, beta = ||r'||^2 / ||r||^2,
// cg.py:125-153): the same IEEE division the host would do, so the coefficient bits do not change.
template <typename T>
__global__ void __launch_bounds__(kBlock) row_ratio_kernel(int64_t rows, const double* __restrict__ num,
                                                           const double* __restrict__ den, T* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += stride) out[i] = (T)(num[i] / den[i]);
}

// ADMM outer update for h = lam ||.||_1, K = Id, and the right-hand side of the next x-update
// (QuadraticFunc.prox -> CG) in one pass (opt/solver/pds.py:1606-1620 + operator.py:1257-1291).  Per element,
// the same functors and the same rounding to T after every step as the chain of map launches it replaces:
//   zt = lincomb3(1, z, 1, x, -1, u)          u' = prox_l1(axpby(1, x, 1, zt), thr)
//   z' = lincomb3(1, zt, rho-1, x, -(rho-1), u')
//   b  = axpby(1, div(axpby(1, u', -1, z'), tau), -1, cgrad)
// Planes of `out` (6 x n): u', z', b, r0 = b, p0 = b, x0 = 0 (CG's start from zero: r0 = b - A 0 = b).
template <typename T>
struct AdmmL1 {
  Lin3Op<T> zt_op;
  AxpbyOp<T> v_op;
  ProxL1Op<T> prox;
  Lin3Op<T> z_op;
  AxpbyOp<T> arr_op;
  DivOp<T> div;
  AxpbyOp<T> b_op;
  __device__ void operator()(T x, T z, T u, T cg, T& un, T& zn, T& b) const {
    const T zt = zt_op(z, x, u);
    un = prox(v_op(x, zt, T(0)), T(0), T(0));
    zn = z_op(zt, x, un);
    b = b_op(div(arr_op(un, zn, T(0)), T(0), T(0)), cg, T(0));
  }
};

template <typename T>
__global__ void __launch_bounds__(kBlock) admm_l1_kernel(int64_t n, AdmmL1<T> op, const T* __restrict__ x,
                                                         const T* __restrict__ z, const T* __restrict__ u,
                                                         const T* __restrict__ cg, T* __restrict__ out, bool vec) {
  constexpr int V = kVecN<T>;
  using VT = typename Vec4<T>::type;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nv = vec ? n / V : 0;
  for (int64_t i = tid; i < nv; i += stride) {
    T vx[V], vz[V], vu[V], vc[V], ou[V], oz[V], ob[V], o0[V];
    *reinterpret_cast<VT*>(vx) = reinterpret_cast<const VT*>(x)[i];
    *reinterpret_cast<VT*>(vz) = reinterpret_cast<const VT*>(z)[i];
    *reinterpret_cast<VT*>(vu) = reinterpret_cast<const VT*>(u)[i];
    *reinterpret_cast<VT*>(vc) = reinterpret_cast<const VT*>(cg)[i];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      op(vx[k], vz[k], vu[k], vc[k], ou[k], oz[k], ob[k]);
      o0[k] = T(0);
    }
    VT* o = reinterpret_cast<VT*>(out);
    const int64_t nq = n / V;
    o[i] = *reinterpret_cast<VT*>(ou);
    o[nq + i] = *reinterpret_cast<VT*>(oz);
    o[2 * nq + i] = *reinterpret_cast<VT*>(ob);
    o[3 * nq + i] = *reinterpret_cast<VT*>(ob);
    o[4 * nq + i] = *reinterpret_cast<VT*>(ob);
    o[5 * nq + i] = *reinterpret_cast<VT*>(o0);
  }
  for (int64_t i = nv * V + tid; i < n; i += stride) {
    T un, zn, b;
    op(x[i], z[i], u[i], cg[i], un, zn, b);
    out[i] = un;
    out[n + i] = zn;
    out[2 * n + i] = b;
    out[3 * n + i] = b;
    out[4 * n + i] = b;
    out[5 * n + i] = T(0);
  }
}

}  // namespace
}  // namespace pxa

using namespace pxa;

extern "C" {

int pxa_admm_l1_update(int dtype, int64_t n, const void* x, const void* z, const void* u, const void* cgrad,
                       double rho_m1, double thr, double tau, void* out, void* stream) {
  PXA_CHECK_ARG(n >= 0);
  if (n == 0) return PXA_OK;
  PXA_CHECK_ARG(x && z && u && cgrad && out);
  PXA_DISPATCH(dtype, T, {
    const T one = T(1), rm = (T)rho_m1;
    const AdmmL1<T> op{Lin3Op<T>{one, one, -one}, AxpbyOp<T>{one, one}, ProxL1Op<T>{(T)thr},
                       Lin3Op<T>{one, rm, -rm},    AxpbyOp<T>{one, -one}, DivOp<T>{(T)tau},
                       AxpbyOp<T>{one, -one}};
    const bool vec = n % kVecN<T> == 0 && aligned16(x) && aligned16(z) && aligned16(u) && aligned16(cgrad) &&
                     aligned16(out);
    const int64_t items = vec ? n / kVecN<T> : n;
    hipLaunchKernelGGL((admm_l1_kernel<T>), dim3(grid_for(items)), dim3(kBlock), 0, as_stream(stream), n, op,
                       (const T*)x, (const T*)z, (const T*)u, (const T*)cgrad, (T*)out, vec);
    return last_launch_status();
  });
}

int pxa_axpby(int dtype, int64_t n, double a, const void* x, double b, const void* y, void* out, void* stream) {
  if (y == nullptr) {
    PXA_DISPATCH(dtype, T, return (launch_map<T, 1>(n, ScaleOp<T>{(T)a}, x, nullptr, nullptr, out, stream)));
  }
  PXA_DISPATCH(dtype, T, return (launch_map<T, 2>(n, AxpbyOp<T>{(T)a, (T)b}, x, y, nullptr, out, stream)));
}

int pxa_axpby_bcast(int dtype, int64_t n, double a, const void* x, double b, const void* y, int64_t ny, void* out,
                    void* stream) {
  PXA_CHECK_ARG(n >= 0 && ny >= 1 && n % ny == 0);
  if (n == 0) return PXA_OK;
  PXA_CHECK_ARG(x && y && out);
  PXA_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((bcast_kernel<T>), dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), n, ny, (T)a,
                       (const T*)x, (T)b, (const T*)y, (T*)out);
    return last_launch_status();
  });
}

int pxa_axpy_rows(int dtype, int64_t rows, int64_t n, const void* c, double s, const void* x, const void* y, void* out,
                  void* stream) {
  PXA_CHECK_ARG(rows >= 0 && n >= 0);
  if (rows * n == 0) return PXA_OK;
  PXA_CHECK_ARG(c && x && y && out);
  PXA_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((axpy_rows_kernel<T>), dim3(grid_for(rows * n)), dim3(kBlock), 0, as_stream(stream), rows, n,
                       (const T*)c, (T)s, (const T*)x, (const T*)y, (T*)out);
    return last_launch_status();
  });
}

int pxa_row_ratio(int dtype, int64_t rows, const double* num, const double* den, void* out, void* stream) {
  PXA_CHECK_ARG(rows >= 0);
  if (rows == 0) return PXA_OK;
  PXA_CHECK_ARG(num && den && out);
  PXA_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((row_ratio_kernel<T>), dim3(grid_for(rows)), dim3(kBlock), 0, as_stream(stream), rows, num, den,
                       (T*)out);
    return last_launch_status();
  });
}

int pxa_lincomb3(int dtype, int64_t n, double a, const void* x, double b, const void* y, double c, const void* z,
                 void* out, void* stream) {
  PXA_DISPATCH(dtype, T, return (launch_map<T, 3>(n, Lin3Op<T>{(T)a, (T)b, (T)c}, x, y, z, out, stream)));
}

int pxa_extrapolate(int dtype, int64_t n, double a, const void* x, const void* y, void* out, void* stream) {
  PXA_DISPATCH(dtype, T, return (launch_map<T, 2>(n, ExtrapOp<T>{(T)a}, x, y, nullptr, out, stream)));
}

int pxa_div(int dtype, int64_t n, const void* x, double d, void* out, void* stream) {
  PXA_DISPATCH(dtype, T, return (launch_map<T, 1>(n, DivOp<T>{(T)d}, x, nullptr, nullptr, out, stream)));
}

int pxa_add_scalar(int dtype, int64_t n, const void* x, double s, void* out, void* stream) {
  PXA_DISPATCH(dtype, T, return (launch_map<T, 1>(n, AddScalarOp<T>{(T)s}, x, nullptr, nullptr, out, stream)));
}

int pxa_mul(int dtype, int64_t n, const void* x, const void* y, void* out, void* stream) {
  PXA_DISPATCH(dtype, T, return (launch_map<T, 2>(n, MulOp<T>{}, x, y, nullptr, out, stream)));
}

int pxa_clip(int dtype, int64_t n, const void* x, double lo, double hi, int has_hi, void* out, void* stream) {
  PXA_DISPATCH(dtype, T,
               return (launch_map<T, 1>(n, ClipOp<T>{(T)lo, (T)hi, has_hi != 0}, x, nullptr, nullptr, out, stream)));
}

int pxa_prox_l1(int dtype, int64_t n, const void* x, double tau, void* out, void* stream) {
  PXA_DISPATCH(dtype, T, return (launch_map<T, 1>(n, ProxL1Op<T>{(T)tau}, x, nullptr, nullptr, out, stream)));
}

int pxa_fenchel_prox_l1(int dtype, int64_t n, const void* x, double sigma, double lam, void* out, void* stream) {
  PXA_DISPATCH(dtype, T, {
    T s = (T)sigma;
    T t = (T(1) / s) * (T)lam;
    return (launch_map<T, 1>(n, FenchelL1Op<T>{s, t}, x, nullptr, nullptr, out, stream));
  });
}

int pxa_moreau_grad_l1(int dtype, int64_t n, const void* x, double mu, double scale, void* out, void* stream) {
  PXA_DISPATCH(dtype, T,
               return (launch_map<T, 1>(n, MoreauL1Op<T>{(T)mu, (T)scale}, x, nullptr, nullptr, out, stream)));
}

int pxa_fill(int dtype, int64_t n, double v, void* out, void* stream) {
  // `a` is read but ignored by FillOp; pass `out` so the pointer is valid and aligned alike.
  PXA_DISPATCH(dtype, T, return (launch_map<T, 1>(n, FillOp<T>{(T)v}, out, nullptr, nullptr, out, stream)));
}

int pxa_prox_l21(int dtype, int64_t outer, int64_t group, int64_t inner, const void* x, double tau, void* out,
                 void* stream) {
  PXA_DISPATCH(dtype, T, return (launch_group<T, kProx>(outer, group, inner, x, out, tau, 0, 0, stream)));
}

int pxa_fenchel_prox_l21(int dtype, int64_t outer, int64_t group, int64_t inner, const void* x, double sigma,
                         double lam, void* out, void* stream) {
  PXA_DISPATCH(dtype, T, {
    T s = (T)sigma;
    T t = (T(1) / s) * (T)lam;
    return (launch_group<T, kFenchel>(outer, group, inner, x, out, (double)s, (double)t, 0, stream));
  });
}

int pxa_moreau_grad_l21(int dtype, int64_t outer, int64_t group, int64_t inner, const void* x, double mu,
                        double scale, void* out, void* stream) {
  PXA_DISPATCH(dtype, T, return (launch_group<T, kMoreau>(outer, group, inner, x, out, mu, 0, scale, stream)));
}

int pxa_group_norm(int dtype, int64_t outer, int64_t group, int64_t inner, const void* x, void* out, void* stream) {
  PXA_DISPATCH(dtype, T, return (launch_group<T, kNorm>(outer, group, inner, x, out, 0, 0, 0, stream)));
}

}  // extern "C"
