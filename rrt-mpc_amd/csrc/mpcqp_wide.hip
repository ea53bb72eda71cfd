// mpcqp_wide.hip -- the solve for long horizons (MPCQP_WIDE_MIN_HORIZON <= N <= MPCQP_MAX_HORIZON).
//
// The one-wave kernel (mpcqp_solve.h) keeps a QP's KKT inverse one row per lane in registers,
// which caps it at 2N <= 62 decision variables.  The reference builds its QP for any horizon
// (src/control/mpc_controller.py:47-57), so longer horizons take this kernel: one 256-thread
// workgroup (four waves) per QP, runtime N, the same algorithm -- condensing, OSQP Ruiz/cost
// scaling, ADMM with adaptive rho and OSQP's termination, the active-set polish -- with every
// array in a per-QP arena: LDS when it fits (N <= ~50), else the workspace in HBM (then L2
// resident); the scaled Hessian Pbar always lives in the workspace.
//
// Arithmetic: this kernel is oracle/mpcqp_cpu.c parallelised without changing a single floating
// point operation -- elementwise work spread over the threads, every sum in the C code's
// sequential order (thread 0 or the owning thread), maxima (exact) reduced in any order, no
// contraction, IEEE division and square root.  Given the same LTV model (K1 output) its
// solutions, statuses and iteration counts equal the C restatement's bit for bit
// (tests/test_gpu_wide.py).
#include "mpcqp_build.h"

namespace {
using mpcqp::Launch;

constexpr int kT = 256;  // threads per QP
constexpr int kTW = kT / kWave;

// ---- arena layout (doubles), offsets from the QP's arena base
struct WideLayout {
  int N, n, m, ks, ps;  // ks / ps: row strides of K / Pbar (n + 1: a column's rows hit distinct banks)
  int oK, oModel, oPa, oPg, oE4, oG, oQ, oD, oX, oXt, oRhs, oPx, oAty, oXp, oXa, oDx, oRes, oPd, oXn, oDl, oCol, oCol2, oCm;
  int oK1, oK2, oEr, oL, oU, oW, oLo0, oHi0, oW0, oZ, oY, oZt, oTmp, oAx, oRw, oZc, oZn, oZd, oEl, oT1, oT2, oCd, oCn,
      oRed, total;
  __host__ __device__ static WideLayout make(int N) {
    WideLayout L{};
    L.N = N;
    L.n = 2 * N;
    L.m = 5 * N;
    L.ks = L.n + 1;
    L.ps = L.n + 1;
    int o = 0;
    auto take = [&](int cnt) {
      const int r = o;
      o += (cnt + 1) / 2 * 2;  // 16-byte alignment
      return r;
    };
    L.oK = take(L.n * L.ks);
    L.oModel = take(model_stride(N));
    L.oPa = take(N + 1);
    L.oPg = take(N + 1);
    L.oE4 = take(4 * (N + 1));
    L.oG = take(L.n + 1);
    L.oQ = take(L.n);
    L.oD = take(L.n);
    L.oX = take(L.n);
    L.oXt = take(L.n);
    L.oRhs = take(L.n);
    L.oPx = take(L.n);
    L.oAty = take(L.n);
    L.oXp = take(L.n);
    L.oXa = take(L.n);
    L.oDx = take(L.n);
    L.oRes = take(L.n);
    L.oPd = take(L.n);
    L.oXn = take(L.n);
    L.oDl = take(L.n);
    L.oCol = take(L.n + 64);  // + padding: the sweep's tail rows read past n
    L.oCol2 = take(L.n + 64);
    L.oCm = take(L.n);
    L.oK1 = take(2 * L.n);
    L.oK2 = take(3 * L.n);
    L.oEr = take(L.m);
    L.oL = take(L.m);
    L.oU = take(L.m);
    L.oW = take(L.m);
    L.oLo0 = take(L.m);
    L.oHi0 = take(L.m);
    L.oW0 = take(L.m);
    L.oZ = take(L.m);
    L.oY = take(L.m);
    L.oZt = take(L.m);
    L.oTmp = take(L.m);
    L.oAx = take(L.m);
    L.oRw = take(L.m);
    L.oZc = take(L.m);
    L.oZn = take(L.m);
    L.oZd = take(L.m);
    L.oEl = take(L.m);
    L.oT1 = take(L.m);
    L.oT2 = take(L.m);
    L.oCd = take(L.m);  // active codes as doubles (0, 1, 2)
    L.oCn = take(L.m);
    L.oRed = take(4 * kTW + 8);
    L.total = o;
    return L;
  }
};

// per-QP workspace doubles: Pbar (n x n) + the arena (used when it does not fit in LDS)
__host__ __device__ inline size_t wide_stride_of(const WideLayout& L) { return (size_t)L.n * L.ps + L.total; }

// ---- block reductions (maxima: exact, any order; flags)
struct Blk {
  double* red;  // 4 * kTW + 8 doubles of the arena
  __device__ double max(double v) const {  // v >= 0 or NaN-free maxima of |.|
    for (int o = kWave / 2; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, kWave));
    __syncthreads();
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = v;
    __syncthreads();
    double r = red[0];
    for (int k = 1; k < kTW; ++k) r = fmax(r, red[k]);
    __syncthreads();
    return r;
  }
  __device__ bool any(bool b) const {
    const bool w = __ballot(b) != 0ull;
    __syncthreads();
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = w ? 1.0 : 0.0;
    __syncthreads();
    bool r = false;
    for (int k = 0; k < kTW; ++k) r = r || red[k] != 0.0;
    __syncthreads();
    return r;
  }
  // sum in tree order (the fast mode's line search; the reproducible mode sums in the C order)
  __device__ double sum(double v) const {
    for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    __syncthreads();
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = v;
    __syncthreads();
    double r = red[0];
    for (int k = 1; k < kTW; ++k) r += red[k];
    __syncthreads();
    return r;
  }
  // thread 0's value to every thread
  __device__ double bcast0(double v) const {
    __syncthreads();
    if (threadIdx.x == 0) red[kTW] = v;
    __syncthreads();
    const double r = red[kTW];
    __syncthreads();
    return r;
  }
};

__device__ __forceinline__ double lim(double v) { return limit_scaling(v); }

// for (e = tid; e < n * n; e += kT) f(e / n, e % n, e) -- the row/column advanced without a
// division per element
template <class F>
__device__ __forceinline__ void for_ij(int n, int tid, F&& f) {
  int i = tid / n, j = tid - (tid / n) * n;
  const int di = kT / n, dj = kT - (kT / n) * n;
  for (int e = tid; e < n * n; e += kT) {
    f(i, j, e);
    i += di;
    j += dj;
    if (j >= n) {
      j -= n;
      ++i;
    }
  }
}

// In-place symmetric sweep K <- K^{-1} (mpcqp_cpu.c sweep_inverse); false on a bad pivot.
// Thread (j, part) keeps rows [part*chunk, +chunk) of column j in registers for all n pivots: per
// pivot the owners of column k publish it (double-buffered, one barrier) and every element is
// updated exactly as the C code does it -- the same operations, no memory traffic for K.  The
// tail rows past n and the idle threads run on copies that are never stored or published, so the
// update is branch-free.  Out of line (its own register allocation, AS: 3 = K in LDS, 1 = in the
// workspace) -- inlined into the solve it drags the whole kernel into spills.
template <int CH, int AS>
__device__ __noinline__ bool sweep_regs(double* Kg, double* c0g, double* c1g, int n, int ks, int tid) {
#pragma clang fp contract(off)
  typedef __attribute__((address_space(AS))) double* Ptr;
  const Ptr Kp = (Ptr)Kg;
  const Ptr cb0 = (Ptr)c0g, cb1 = (Ptr)c1g;
  const int per = kT / n;  // threads per column (>= 2: n <= 126)
  const int j = tid % n, part = tid / n;
  const int chunk = (n + per - 1) / per;
  const bool own = part < per;
  const int i0 = own ? part * chunk : 0;
  double R[CH];
#pragma unroll
  for (int r = 0; r < CH; ++r) R[r] = Kp[(size_t)min(i0 + r, n - 1) * ks + j];
  for (int k = 0; k < n; ++k) {
    const Ptr col = (k & 1) ? cb1 : cb0;  // (a two-element array here would live in scratch)
    if (own && j == k) {
#pragma unroll
      for (int r = 0; r < CH; ++r)
        if (r < chunk && i0 + r < n) col[i0 + r] = R[r];
    }
    __syncthreads();
    const double d = col[k];
    const double cj = col[j];
    const Ptr ci = col + i0;  // rows i0 .. i0 + CH - 1 (the buffers are padded past n)
    constexpr int G = CH < 16 ? CH : 16;  // rows whose column values are in flight at once
    double cv[G];
#pragma unroll
    for (int r = 0; r < G; ++r) cv[r] = ci[r];  // issued before the division they overlap
    __builtin_amdgcn_sched_barrier(0);
    if (!(d > 0.0) || !isfinite(d)) return false;  // uniform: every thread reads the same pivot
    const double inv = 1.0 / d;
    const double cjk = cj * inv;
    const bool jk = j == k;
#pragma unroll
    for (int g = 0; g < CH; g += G) {
      if (g) {
#pragma unroll
        for (int r = 0; r < G; ++r) cv[r] = ci[g + r];
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int r = 0; r < G; ++r) {  // rows i != k (both arms use the load: no branch per row)
        const double f = cv[r] * inv;
        R[g + r] = jk ? f : R[g + r] - f * cj;
      }
    }
    const double rowk = jk ? -inv : cjk;
    const int rk = k - i0;
#pragma unroll
    for (int r = 0; r < CH; ++r) R[r] = r == rk ? rowk : R[r];  // row k: cheap selects
  }
  if (own) {
#pragma unroll
    for (int r = 0; r < CH; ++r)
      if (r < chunk && i0 + r < n) Kp[(size_t)(i0 + r) * ks + j] = -R[r];
  }
  __syncthreads();
  return true;
}

// The per-QP state of the wide solve: pointers into the arena + the workspace Pbar.
struct Wide {
  WideLayout L;
  double* A;   // arena
  bool in_lds;  // the arena is in LDS (a compile-time constant of the kernel)
  double* P;   // Pbar, n x n row-major (workspace)
  Blk blk;
  int tid;
  double c;    // cost scaling (uniform)
  double dt;
#ifdef MPCQP_WIDE_STAMPS  // diagnostic builds: per-phase s_memtime sums of thread 0 -> st[0..15]
  double* st = nullptr;
  unsigned long long t_last = 0;
  __device__ void mark() { if (tid == 0) t_last = __builtin_amdgcn_s_memtime(); }
  __device__ void stamp(int slot) {
    if (tid == 0 && st) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      st[slot] += (double)(t - t_last);
      t_last = t;
    }
  }
#else
  __device__ void mark() {}
  __device__ void stamp(int) {}
#endif
  __device__ double* at(int off) const { return A + off; }
  __device__ double& K(int i, int j) const { return A[L.oK + i * L.ks + j]; }

  // z = Cbar x (mpcqp_cpu.c Cmul)
  __device__ void Cmul(const double* x, double* z) const {
#pragma clang fp contract(off)
    const int N = L.N, n = L.n;
    const double* D = at(L.oD);
    const double* E = at(L.oEr);
    const double* k1 = at(L.oK1);
    const double* k2 = at(L.oK2);
    __syncthreads();
    for (int j = tid; j < N; j += kT) z[j] = E[j] * (D[2 * j] * x[2 * j]);
    for (int p = tid; p < n; p += kT) {
      const double e1 = E[N + p], e2 = E[3 * N + p];
      const double t0 = D[p] * x[p];
      const double tm2 = p >= 2 ? D[p - 2] * x[p - 2] : 0.0;
      const double tm4 = p >= 4 ? D[p - 4] * x[p - 4] : 0.0;
      z[N + p] = (e1 * k1[2 * p]) * t0 + (e1 * k1[2 * p + 1]) * tm2;
      z[3 * N + p] = ((e2 * k2[3 * p]) * t0 + (e2 * k2[3 * p + 1]) * tm2) + (e2 * k2[3 * p + 2]) * tm4;
    }
    __syncthreads();
  }
  // x = Cbar' y (mpcqp_cpu.c CTmul)
  __device__ void CTmul(const double* y, double* x) const {
#pragma clang fp contract(off)
    const int N = L.N, n = L.n;
    const double* D = at(L.oD);
    const double* E = at(L.oEr);
    const double* k1 = at(L.oK1);
    const double* k2 = at(L.oK2);
    __syncthreads();
    for (int p = tid; p < n; p += kT) {
      const double e1 = E[N + p], e2 = E[3 * N + p];
      double t = ((p & 1) == 0 ? E[p / 2] * y[p / 2] : 0.0) + (e1 * k1[2 * p]) * y[N + p];
      t += (e2 * k2[3 * p]) * y[3 * N + p];
      double a1 = 0.0, b2 = 0.0;  // a1[p + 2], b2[p + 4] of the C code
      if (p + 2 < n) {
        const double f1 = E[N + p + 2], f2 = E[3 * N + p + 2];
        a1 = (f1 * k1[2 * (p + 2) + 1]) * y[N + p + 2] + (f2 * k2[3 * (p + 2) + 1]) * y[3 * N + p + 2];
      }
      if (p + 4 < n) b2 = (E[3 * N + p + 4] * k2[3 * (p + 4) + 2]) * y[3 * N + p + 4];
      t += a1;
      t += b2;
      x[p] = D[p] * t;
    }
    __syncthreads();
  }
  // y = M x, M row-major with row stride ms (thread i: the C code's sequential row sum; the loads
  // run ahead of the sum in groups of 8)
  __device__ void matvec(const double* M, int ms, const double* x, double* y) const {
#pragma clang fp contract(off)
    __syncthreads();
    const double* __restrict__ xr = x;
    for (int i = tid; i < L.n; i += kT) {
      const double* __restrict__ row = M + (size_t)i * ms;
      double t = 0.0;
#pragma unroll 8
      for (int j = 0; j < L.n; ++j) t += row[j] * xr[j];
      y[i] = t;
    }
    __syncthreads();
  }
  // (Pbar + sig I + D (Cbar' diag(rw) Cbar)_band D)[i][j]  (mpcqp_cpu.c form_kkt: the band entry
  // Bd[i][j] accumulated in the C code's order -- the v row, then rows p = max(i, j), +2, +4,
  // slot 1 before slot 2 of each)
  __device__ double kkt(int i, int j, double sig, const double* rw) const {
#pragma clang fp contract(off)
    const int N = L.N, n = L.n;
    const double* D = at(L.oD);
    const double* E = at(L.oEr);
    const double* k1 = at(L.oK1);
    const double* k2 = at(L.oK2);
    double bd = 0.0;
    const int dij = i > j ? i - j : j - i;
    if ((dij & 1) == 0 && dij <= 4) {
      if (i == j && (i & 1) == 0) bd += E[i / 2] * E[i / 2] * rw[i / 2];
      const int pm = i > j ? i : j, pl = i > j ? j : i;
      for (int p = pm; p <= pl + 4 && p < n; p += 2) {
        const int a = (p - i) / 2, b = (p - j) / 2;  // coefficient a multiplies variable p - 2a = i
        const double e1 = E[N + p], e2 = E[3 * N + p];
        if (a < 2 && b < 2) {
          const double ca = e1 * k1[2 * p + a], cb = e1 * k1[2 * p + b];
          if (ca != 0.0 && cb != 0.0) bd += rw[N + p] * ca * cb;
        }
        const double ca = e2 * k2[3 * p + a], cb = e2 * k2[3 * p + b];
        if (ca != 0.0 && cb != 0.0) bd += rw[3 * N + p] * ca * cb;
      }
    }
    return P[(size_t)i * L.ps + j] + D[i] * D[j] * bd + (i == j ? sig : 0.0);
  }
  __device__ void form(double sig, const double* rw) const {
    const int n = L.n;
    __syncthreads();
    for_ij(n, tid, [&](int i, int j, int e) {
      K(i, j) = kkt(i, j, sig, rw);
    });
    __syncthreads();
  }
  // y = M x for the Newton matrix M = kkt(., ., 0, rw) (the C code's matvec over its stored M)
  __device__ void kkt_matvec(const double* rw, const double* x, double* y) const {
#pragma clang fp contract(off)
    __syncthreads();
    for (int i = tid; i < L.n; i += kT) {
      double t = 0.0;
      for (int j = 0; j < L.n; ++j) t += kkt(i, j, 0.0, rw) * x[j];
      y[i] = t;
    }
    __syncthreads();
  }
  // The C code's sweep_inverse on K where it lives (n > 128: a column does not fit the
  // register-resident sweep's 64 rows per thread): per pivot the column is copied, then every
  // element updated exactly as the C code updates it, one barrier per pivot.
  __device__ __forceinline__ bool sweep_mem() const {
#pragma clang fp contract(off)
    const int n = L.n;
    double* col = A + L.oCol;
    for (int k = 0; k < n; ++k) {
      __syncthreads();
      for (int i = tid; i < n; i += kT) col[i] = K(i, k);
      __syncthreads();
      const double d = col[k];
      if (!(d > 0.0) || !isfinite(d)) return false;  // uniform
      const double inv = 1.0 / d;
      for_ij(n, tid, [&](int i, int j, int) {
        if (i == k)
          K(k, j) = j == k ? -inv : col[j] * inv;
        else if (j == k)
          K(i, k) = col[i] * inv;
        else
          K(i, j) = K(i, j) - (col[i] * inv) * col[j];
      });
    }
    __syncthreads();
    for_ij(n, tid, [&](int i, int j, int) { K(i, j) = -K(i, j); });  // A holds -A^{-1}
    __syncthreads();
    return true;
  }
  __device__ __forceinline__ bool sweep() const {
    const int per = kT / L.n;  // threads per column (0 past 2N = 256)
    if (per == 0 || (L.n + per - 1) / per > 64) return sweep_mem();
    const int chunk = (L.n + per - 1) / per;
    double *Kp = A + L.oK, *c0 = A + L.oCol, *c1 = A + L.oCol2;
    if (in_lds) {
      if (chunk <= 16) return sweep_regs<16, 3>(Kp, c0, c1, L.n, L.ks, tid);
      if (chunk <= 32) return sweep_regs<32, 3>(Kp, c0, c1, L.n, L.ks, tid);
      return sweep_regs<64, 3>(Kp, c0, c1, L.n, L.ks, tid);
    }
    if (chunk <= 16) return sweep_regs<16, 1>(Kp, c0, c1, L.n, L.ks, tid);
    if (chunk <= 32) return sweep_regs<32, 1>(Kp, c0, c1, L.n, L.ks, tid);
    return sweep_regs<64, 1>(Kp, c0, c1, L.n, L.ks, tid);
  }
  // K <- kkt(., ., sig, rw)^{-1} (form_kkt + sweep_inverse of the C code)
  __device__ __forceinline__ bool form_inverse(double sig, const double* rw) const {
    form(sig, rw);
    return sweep();
  }
  __device__ static int code(double z, double l, double u) { return z > u ? 2 : (z < l ? 1 : 0); }
  // Fast mode's polish: Sherman-Morrison on K = A^{-1} for A' = A + delta c c', c the scaled row r
  // of Cbar (at most three entries: Cmul's coefficients).  K' = K - kap u u', u = K c (three
  // columns of K), kap = delta / (1 + delta c'u).  false (K untouched) when the denominator is not
  // safely positive -- the caller refactorizes.
  __device__ bool rank1(int r, double delta) const {
    const int N = L.N, n = L.n;
    const double* D = at(L.oD);
    const double* E = at(L.oEr);
    const double* k1 = at(L.oK1);
    const double* k2 = at(L.oK2);
    int idx[3] = {0, 0, 0};
    double cf[3] = {0.0, 0.0, 0.0};
    if (r < N) {
      idx[0] = 2 * r;
      cf[0] = E[r] * D[2 * r];
    } else if (r < 3 * N) {
      const int p = r - N;
      for (int a = 0; a < 2; ++a)
        if (p - 2 * a >= 0) {
          idx[a] = p - 2 * a;
          cf[a] = (E[r] * k1[2 * p + a]) * D[p - 2 * a];
        }
    } else {
      const int p = r - 3 * N;
      for (int a = 0; a < 3; ++a)
        if (p - 2 * a >= 0) {
          idx[a] = p - 2 * a;
          cf[a] = (E[r] * k2[3 * p + a]) * D[p - 2 * a];
        }
    }
    double* uv = at(L.oCm);
    __syncthreads();
    for (int i = tid; i < n; i += kT) uv[i] = (cf[0] * K(i, idx[0]) + cf[1] * K(i, idx[1])) + cf[2] * K(i, idx[2]);
    __syncthreads();
    const double cu = (cf[0] * uv[idx[0]] + cf[1] * uv[idx[1]]) + cf[2] * uv[idx[2]];
    const double den = 1.0 + delta * cu;
    if (!(den > kRank1Min) || !isfinite(den)) return false;  // uniform: every thread, same values
    const double kap = delta / den;
    for_ij(n, tid, [&](int i, int j, int) { K(i, j) -= (kap * uv[i]) * uv[j]; });
    __syncthreads();
    return true;
  }
};

// condensing + scaling (mpcqp_cpu.c condense + setup_qp); returns bad (non-finite data)
__device__ bool wide_setup(const mpcqp_params& p, Wide& S) {
#pragma clang fp contract(off)
  const WideLayout& L = S.L;
  const int N = L.N, n = L.n, m = L.m, tid = S.tid;
  const double* mdl = S.at(L.oModel);
  const double* al = mdl;
  const double* be = mdl + N;
  const double* ga = mdl + 2 * N;
  const double* et = mdl + 3 * N;
  const double* si = mdl + 4 * N;
  const double* c0 = mdl + 5 * N;
  const double* c1 = mdl + 6 * N;
  const double* r = mdl + 7 * N;
  const double* x0 = mdl + 11 * N + 4;
  const double* up = mdl + 11 * N + 8;
  const double dt = p.dt;
  double* Pa = S.at(L.oPa);
  double* Pg = S.at(L.oPg);
  double* e4 = S.at(L.oE4);
  double* g = S.at(L.oG);
  if (tid == 0) {
    Pa[0] = Pg[0] = 0.0;
    for (int k = 0; k < N; ++k) {
      Pa[k + 1] = Pa[k] + al[k];
      Pg[k + 1] = Pg[k] + ga[k];
    }
  } else if (tid == kWave) {  // free response, another wave
    double px = x0[0], py = x0[1];
    const double psi = x0[2];
    for (int mm = 1; mm <= N; ++mm) {
      const int k = mm - 1;
      const double v = k == 0 ? x0[3] : 0.0;
      px = px + al[k] * psi + be[k] * v + c0[k];
      py = py + ga[k] * psi + et[k] * v + c1[k];
      e4[4 * mm + 0] = px - r[4 * mm + 0];
      e4[4 * mm + 1] = py - r[4 * mm + 1];
      e4[4 * mm + 2] = psi - r[4 * mm + 2];
      e4[4 * mm + 3] = 0.0 - r[4 * mm + 3];
    }
  }
  __syncthreads();
  double Q[4][4], QN[4][4], R[2][2];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      Q[i][j] = 0.5 * (p.q[4 * i + j] + p.q[4 * j + i]);
      QN[i][j] = 0.5 * (p.q_terminal[4 * i + j] + p.q_terminal[4 * j + i]);
    }
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) R[i][j] = 0.5 * (p.r[2 * i + j] + p.r[2 * j + i]);
  // column `col` of H (the workspace P buffer holds H until P = 2H), col == n -> g
  for (int col = tid; col <= n; col += kT) {
    const int j = col >> 1, cc = col & 1;
    double mu[3] = {0, 0, 0};
    for (int mm = N; mm >= 1; --mm) {
      double sv[4];
      if (col == n) {
        sv[0] = e4[4 * mm + 0];
        sv[1] = e4[4 * mm + 1];
        sv[2] = e4[4 * mm + 2];
        sv[3] = e4[4 * mm + 3];
      } else if (cc == 0) {
        const bool on = mm >= j + 2;
        sv[0] = on ? be[j + 1] : 0.0;
        sv[1] = on ? et[j + 1] : 0.0;
        sv[2] = 0.0;
        sv[3] = mm == j + 1 ? 1.0 : 0.0;
      } else if (mm > j) {
        sv[0] = si[j] * (Pa[mm] - Pa[j + 1]);
        sv[1] = si[j] * (Pg[mm] - Pg[j + 1]);
        sv[2] = si[j];
        sv[3] = 0.0;
      } else {
        sv[0] = sv[1] = sv[2] = sv[3] = 0.0;
      }
      const bool term = mm == N;
      double ws[4];
      for (int a = 0; a < 4; ++a) {
        const double* W = term ? QN[a] : Q[a];
        ws[a] = W[0] * sv[0] + W[1] * sv[1] + W[2] * sv[2] + W[3] * sv[3];
      }
      double hv;
      if (mm < N) {
        const double m0 = mu[0], m1 = mu[1];
        hv = ws[3] + (be[mm] * m0 + et[mm] * m1);
        mu[0] = ws[0] + m0;
        mu[1] = ws[1] + m1;
        mu[2] = ws[2] + (mu[2] + al[mm] * m0 + ga[mm] * m1);
      } else {
        hv = ws[3];
        mu[0] = ws[0];
        mu[1] = ws[1];
        mu[2] = ws[2];
      }
      const double hd = si[mm - 1] * mu[2];
      if (col == n) {
        g[2 * (mm - 1)] = hv;
        g[2 * (mm - 1) + 1] = hd;
      } else {
        S.P[(size_t)(2 * (mm - 1)) * L.ps + col] = hv;
        S.P[(size_t)(2 * (mm - 1) + 1) * L.ps + col] = hd;
      }
    }
    const double r00 = R[0][0] / (dt * dt), r10 = R[1][0] / dt;
    double* H = S.P;
    if (col == n) {
      g[0] += -x0[3] * r00;
      g[1] += -x0[3] * r10;
    } else if (cc == 0) {
      H[(size_t)col * L.ps + col] += j + 1 < N ? 2.0 * r00 : r00;
      if (j >= 1) H[(size_t)(col - 2) * L.ps + col] += -r00;
      if (j + 1 < N) H[(size_t)(col + 2) * L.ps + col] += -r00;
      H[(size_t)(col + 1) * L.ps + col] += r10;
      if (j + 1 < N) H[(size_t)(col + 3) * L.ps + col] += -r10;
    } else {
      H[(size_t)(col - 1) * L.ps + col] += r10;
      if (j >= 1) H[(size_t)(col - 3) * L.ps + col] += -r10;
      H[(size_t)col * L.ps + col] += R[1][1];
    }
  }
  __syncthreads();
  double* q = S.at(L.oQ);
  double* D = S.at(L.oD);
  double* E = S.at(L.oEr);
  double* k1 = S.at(L.oK1);
  double* k2 = S.at(L.oK2);
  double* lo0 = S.at(L.oLo0);
  double* hi0 = S.at(L.oHi0);
  double* w0 = S.at(L.oW0);
  for_ij(n, tid, [&](int i, int j, int) { S.P[(size_t)i * L.ps + j] = 2.0 * S.P[(size_t)i * L.ps + j]; });
  const double idt = 1.0 / p.dt, v0 = x0[3];
  for (int i = tid; i < n; i += kT) {
    q[i] = 2.0 * g[i];
    if ((i & 1) == 0) {
      k1[2 * i] = idt;
      k1[2 * i + 1] = i >= 2 ? -idt : 0.0;
      k2[3 * i] = idt;
      k2[3 * i + 1] = i >= 2 ? -2.0 * idt : 0.0;
      k2[3 * i + 2] = i >= 4 ? idt : 0.0;
    } else {
      k1[2 * i] = 1.0;
      k1[2 * i + 1] = 0.0;
      k2[3 * i] = 1.0;
      k2[3 * i + 1] = i >= 3 ? -1.0 : 0.0;
      k2[3 * i + 2] = 0.0;
    }
    const int c = i & 1;
    const double ofa = i == 0 ? v0 * idt : 0.0;
    const double ofr = i < 2 ? up[c] + ofa : (i == 2 ? -v0 * idt : 0.0);
    lo0[N + i] = p.u_bounds[2 * c] + ofa;
    hi0[N + i] = p.u_bounds[2 * c + 1] + ofa;
    w0[N + i] = p.slack_input;
    lo0[3 * N + i] = p.du_bounds[2 * c] + ofr;
    hi0[3 * N + i] = p.du_bounds[2 * c + 1] + ofr;
    w0[3 * N + i] = p.slack_rate;
    D[i] = 1.0;
  }
  for (int j = tid; j < N; j += kT) {
    lo0[j] = p.v_bounds[0];
    hi0[j] = p.v_bounds[1];
    w0[j] = p.slack_velocity;
  }
  for (int rr = tid; rr < m; rr += kT) E[rr] = 1.0;
  __syncthreads();
  double* dl = S.at(L.oDl);
  double* el = S.at(L.oEl);
  double* cm = S.at(L.oCm);
  double c = 1.0, cpend = 1.0;
  for (int it = 0; it < p.scaling; ++it) {
    for (int qq = tid; qq < n; qq += kT) {
      double cp = 0.0;
#pragma unroll 8
      for (int i = 0; i < n; ++i) cp = fmax(cp, fabs(S.P[(size_t)i * L.ps + qq]));
      cp *= cpend;
      double cc = (qq & 1) == 0 ? E[qq / 2] : 0.0;
      cc = fmax(cc, E[N + qq] * fabs(k1[2 * qq]));
      cc = fmax(cc, E[3 * N + qq] * fabs(k2[3 * qq]));
      if (qq + 2 < n) {
        cc = fmax(cc, E[N + qq + 2] * fabs(k1[2 * (qq + 2) + 1]));
        cc = fmax(cc, E[3 * N + qq + 2] * fabs(k2[3 * (qq + 2) + 1]));
      }
      if (qq + 4 < n) cc = fmax(cc, E[3 * N + qq + 4] * fabs(k2[3 * (qq + 4) + 2]));
      cc *= D[qq];
      dl[qq] = 1.0 / sqrt(lim(fmax(cp, cc)));
      const double dm2 = qq >= 2 ? D[qq - 2] : 0.0, dm4 = qq >= 4 ? D[qq - 4] : 0.0;
      const double r1 = fmax(fabs(k1[2 * qq]) * D[qq], fabs(k1[2 * qq + 1]) * dm2);
      const double r2 = fmax(fmax(fabs(k2[3 * qq]) * D[qq], fabs(k2[3 * qq + 1]) * dm2), fabs(k2[3 * qq + 2]) * dm4);
      el[N + qq] = 1.0 / sqrt(lim(E[N + qq] * r1));
      el[3 * N + qq] = 1.0 / sqrt(lim(E[3 * N + qq] * r2));
    }
    for (int j = tid; j < N; j += kT) el[j] = 1.0 / sqrt(lim(E[j] * D[2 * j]));
    __syncthreads();
    for_ij(n, tid, [&](int i, int j, int e) {
      const double dlc = dl[j] * cpend;
      S.P[(size_t)i * L.ps + j] = S.P[(size_t)i * L.ps + j] * (dl[i] * dlc);
    });
    for (int i = tid; i < n; i += kT) {
      D[i] *= dl[i];
      q[i] *= dl[i];
    }
    for (int rr = tid; rr < m; rr += kT) E[rr] *= el[rr];
    __syncthreads();
    double qm = 0.0;
    for (int qq = tid; qq < n; qq += kT) {
      double cp = 0.0;
#pragma unroll 8
      for (int i = 0; i < n; ++i) cp = fmax(cp, fabs(S.P[(size_t)i * L.ps + qq]));
      cm[qq] = cp;
      qm = fmax(qm, fabs(q[qq]));
    }
    qm = S.blk.max(qm);  // synchronizes: cm complete
    double cn = 0.0;
#pragma unroll 8
    for (int qq = 0; qq < n; ++qq) cn += cm[qq];  // every thread, the C code's order
    cn /= n;
    const double ct = 1.0 / lim(fmax(cn, lim(qm)));
    cpend = ct;
    for (int i = tid; i < n; i += kT) q[i] *= ct;
    c *= ct;
    __syncthreads();
  }
  for_ij(n, tid, [&](int i, int j, int) { S.P[(size_t)i * L.ps + j] *= cpend; });
  double* l = S.at(L.oL);
  double* u = S.at(L.oU);
  double* w = S.at(L.oW);
  for (int rr = tid; rr < m; rr += kT) {
    l[rr] = E[rr] * lo0[rr];
    u[rr] = E[rr] * hi0[rr];
    w[rr] = c * w0[rr] / (E[rr] * E[rr]);
  }
  S.c = c;
  __syncthreads();
  bool bad = false;
  for (int i = tid; i < n; i += kT) bad = bad || !isfinite(q[i]);
  for_ij(n, tid, [&](int i, int j, int) { bad = bad || !isfinite(S.P[(size_t)i * L.ps + j]); });
  for (int rr = tid; rr < m; rr += kT) bad = bad || !isfinite(l[rr]) || !isfinite(u[rr]);
  return S.blk.any(bad);
}

// mpcqp_cpu.c polish_run: 1 exact optimum found (x = it), 0 not within max_it passes, -1 failure
// FAST (reproducible = 0, N >= MPCQP_WIDE_MIN_HORIZON): passes after the first update the
// inverse by rank-1 changes of the rows that entered or left the set (a full form + sweep when
// more than n/2 changed or an update is unsafe), and the line search's sums run in tree order --
// the one-wave kernel's polish.  Otherwise every pass refactorizes and sums run in the C order.
template <bool FAST>
__device__ int wide_polish(Wide& S, double* x, const double* zg, int max_it, int& pol_it, int& n_fact, int& n_ls) {
#pragma clang fp contract(off)
  const WideLayout& L = S.L;
  const int n = L.n, m = L.m, tid = S.tid;
  const double* q = S.at(L.oQ);
  const double* l = S.at(L.oL);
  const double* u = S.at(L.oU);
  const double* w = S.at(L.oW);
  double* cd = S.at(L.oCd);
  double* cn = S.at(L.oCn);
  double* zc = S.at(L.oZc);
  double* rw = S.at(L.oRw);
  double* tmp = S.at(L.oTmp);
  double* rhs = S.at(L.oRhs);
  double* xn = S.at(L.oXn);
  double* zn = S.at(L.oZn);
  double* res = S.at(L.oRes);
  double* dx = S.at(L.oDx);
  double* Px = S.at(L.oPx);
  double* Pd = S.at(L.oPd);
  double* zd = S.at(L.oZd);
  double* t1 = S.at(L.oT1);
  double* t2 = S.at(L.oT2);
  double* rwf = S.at(L.oEl);  // FAST: soft-row weights of the current factorization (setup scratch)
  double* chg = S.at(L.oT1);  // FAST: rows whose weight changed (the line search's scratch otherwise)
  bool have_fact = false;
  S.Cmul(x, zc);
  S.matvec(S.P, L.ps, x, Px);
  for (int r = tid; r < m; r += kT) cd[r] = Wide::code(zg[r], l[r], u[r]);
  __syncthreads();
  for (int it = 1; it <= max_it; ++it) {
    ++pol_it;
    for (int r = tid; r < m; r += kT) {
      rw[r] = cd[r] != 0.0 ? 2.0 * w[r] : 0.0;
      tmp[r] = cd[r] == 2.0 ? rw[r] * u[r] : (cd[r] == 1.0 ? rw[r] * l[r] : 0.0);
    }
    S.mark();
    ++n_fact;
    bool refac = true;
    if (FAST && have_fact) {
      __syncthreads();
      int nchg = 0;
      if (tid == 0)
        for (int r = 0; r < m; ++r)
          if (rw[r] != rwf[r]) chg[nchg++] = (double)r;
      nchg = (int)S.blk.bcast0((double)nchg);
      refac = nchg > n / 2;
      for (int k = 0; k < nchg && !refac; ++k) {
        const int r = (int)chg[k];
        refac = !S.rank1(r, rw[r] - rwf[r]);
      }
    }
    if (refac) {
      if (!S.form_inverse(0.0, rw)) return -1;
      have_fact = true;
    }
    if (FAST) {
      for (int r = tid; r < m; r += kT) rwf[r] = rw[r];
      __syncthreads();
    }
    S.stamp(5);
    S.CTmul(tmp, rhs);
    for (int i = tid; i < n; i += kT) rhs[i] -= q[i];
    S.matvec(&S.K(0, 0), L.ks, rhs, xn);
    S.Cmul(xn, zn);
    bool nf = false, diff = false;
    for (int i = tid; i < n; i += kT) nf = nf || !isfinite(xn[i]);
    for (int r = tid; r < m; r += kT) diff = diff || Wide::code(zn[r], l[r], u[r]) != cd[r];
    if (S.blk.any(nf)) return -1;
    S.stamp(6);
    if (!S.blk.any(diff)) {
      // the set reproduces itself: one step of iterative refinement, then accept if it still does
      S.kkt_matvec(rw, xn, res);
      for (int i = tid; i < n; i += kT) res[i] = rhs[i] - res[i];
      S.matvec(&S.K(0, 0), L.ks, res, dx);
      for (int i = tid; i < n; i += kT) xn[i] += dx[i];
      S.Cmul(xn, zn);
      nf = false;
      diff = false;
      for (int i = tid; i < n; i += kT) nf = nf || !isfinite(xn[i]);
      for (int r = tid; r < m; r += kT) diff = diff || Wide::code(zn[r], l[r], u[r]) != cd[r];
      if (S.blk.any(nf)) return -1;
      if (!S.blk.any(diff)) {
        for (int i = tid; i < n; i += kT) x[i] = xn[i];
        __syncthreads();
        return 1;
      }
    }
    // exact line search along d = xn - x (P xn from the Newton system, no product with P)
    for (int r = tid; r < m; r += kT)
      tmp[r] = rw[r] * (zn[r] - (cd[r] == 2.0 ? u[r] : (cd[r] == 1.0 ? l[r] : 0.0)));
    S.CTmul(tmp, Pd);
    for (int i = tid; i < n; i += kT) {
      dx[i] = xn[i] - x[i];
      Pd[i] = (-Pd[i] - q[i]) - Px[i];
    }
    for (int r = tid; r < m; r += kT) zd[r] = zn[r] - zc[r];
    __syncthreads();
    double qd = 0.0, lin = 0.0;
    if constexpr (FAST) {
      double a = 0.0, c = 0.0;
      for (int i = tid; i < n; i += kT) {
        a += dx[i] * Pd[i];
        c += (Px[i] + q[i]) * dx[i];
      }
      qd = S.blk.sum(a);
      lin = S.blk.sum(c);
    } else {
#pragma unroll 8
      for (int i = 0; i < n; ++i) {  // every thread, the C code's order
        qd += dx[i] * Pd[i];
        lin += (Px[i] + q[i]) * dx[i];
      }
    }
    double t = 1.0;
    for (int ls = 0; ls < 40; ++ls) {
      ++n_ls;
      double d1 = lin + t * qd, d2 = qd;
      if constexpr (FAST) {
        double a = 0.0, c = 0.0;
        for (int r = tid; r < m; r += kT) {
          const double zt = zc[r] + t * zd[r];
          const double rr = zt > u[r] ? zt - u[r] : (zt < l[r] ? zt - l[r] : 0.0);
          a += 2.0 * w[r] * rr * zd[r];
          if (rr != 0.0) c += 2.0 * w[r] * zd[r] * zd[r];
        }
        d1 += S.blk.sum(a);
        d2 += S.blk.sum(c);
      } else {
        for (int r = tid; r < m; r += kT) {
          const double zt = zc[r] + t * zd[r];
          const double rr = zt > u[r] ? zt - u[r] : (zt < l[r] ? zt - l[r] : 0.0);
          t1[r] = 2.0 * w[r] * rr * zd[r];
          t2[r] = rr != 0.0 ? 2.0 * w[r] * zd[r] * zd[r] : -1.0;  // -1: not added (the term is >= 0)
        }
        __syncthreads();
#pragma unroll 8
        for (int r = 0; r < m; ++r) {  // the C code's order; d2 takes the rows with rr != 0 only
          d1 += t1[r];
          if (t2[r] >= 0.0) d2 += t2[r];
        }
        __syncthreads();
      }
      if (d1 <= 0.0 || !(d2 > 0.0)) break;
      const double tn = fmax(0.0, t - d1 / d2);
      if (tn >= t) break;
      bool moved = false;
      for (int r = tid; r < m; r += kT) {
        const double za = zc[r] + t * zd[r], zb = zc[r] + tn * zd[r];
        moved = moved || Wide::code(za, l[r], u[r]) != Wide::code(zb, l[r], u[r]);
      }
      t = tn;
      if (!S.blk.any(moved)) break;
    }
    for (int i = tid; i < n; i += kT) {
      x[i] += t * dx[i];
      Px[i] += t * Pd[i];
    }
    S.Cmul(x, zc);
    for (int r = tid; r < m; r += kT) cd[r] = Wide::code(zc[r], l[r], u[r]);
    __syncthreads();
    S.stamp(7);
  }
  return 0;
}

// mpcqp_cpu.c mpcqp_cpu_solve_one after setup: ADMM (+ early polish), final polish, outputs
template <bool FAST>
__device__ void wide_solve(const mpcqp_params& p, Wide& S, bool bad, int b, double* __restrict__ u0o,
                           double* __restrict__ Xo, double* __restrict__ Uo, int32_t* __restrict__ statuso,
                           int32_t* __restrict__ iterso, uint8_t* __restrict__ activeo) {
#pragma clang fp contract(off)
  const WideLayout& L = S.L;
  const int N = L.N, n = L.n, m = L.m, tid = S.tid;
  const double* q = S.at(L.oQ);
  const double* D = S.at(L.oD);
  const double* E = S.at(L.oEr);
  const double* l = S.at(L.oL);
  const double* u = S.at(L.oU);
  const double* w = S.at(L.oW);
  double* x = S.at(L.oX);
  double* xt = S.at(L.oXt);
  double* rhs = S.at(L.oRhs);
  double* z = S.at(L.oZ);
  double* y = S.at(L.oY);
  double* zt = S.at(L.oZt);
  double* tmp = S.at(L.oTmp);
  double* Ax = S.at(L.oAx);
  double* Px = S.at(L.oPx);
  double* Aty = S.at(L.oAty);
  double* xp = S.at(L.oXp);
  double* xa = S.at(L.oXa);
  double* rw = S.at(L.oRw);
  for (int i = tid; i < n; i += kT) x[i] = 0.0;
  for (int r = tid; r < m; r += kT) z[r] = y[r] = 0.0;
  __syncthreads();
  int st = MPCQP_MAX_ITER_REACHED;
  int admm_it = 0, pol_it = 0, n_fact = 0, n_ls = 0;
  bool admm_ok = false, polished = false, approx = false;
  if (p.method == MPCQP_METHOD_ADMM) {
    double rho = p.rho;
    const double sig = p.sigma, a = p.alpha;
    bool refactor = true;
    for (int it = 1; it <= p.max_iter && !bad; ++it) {
      S.mark();
      if (refactor) {
        for (int r = tid; r < m; r += kT) rw[r] = rho;
        ++n_fact;
        if (!S.form_inverse(sig, rw)) {
          bad = true;
          break;
        }
        refactor = false;
        S.stamp(1);
      }
      for (int r = tid; r < m; r += kT) tmp[r] = rho * z[r] - y[r];
      S.CTmul(tmp, rhs);
      for (int i = tid; i < n; i += kT) rhs[i] += sig * x[i] - q[i];
      S.matvec(&S.K(0, 0), L.ks, rhs, xt);
      S.Cmul(xt, zt);
      for (int i = tid; i < n; i += kT) x[i] = a * xt[i] + (1.0 - a) * x[i];
      const double ir = 1.0 / rho;
      for (int r = tid; r < m; r += kT) {
        const double v = a * zt[r] + (1.0 - a) * z[r];
        const double vv = v + y[r] * ir;
        double zn = vv;
        if (vv > u[r])
          zn = (rho * vv + 2.0 * w[r] * u[r]) / (rho + 2.0 * w[r]);
        else if (vv < l[r])
          zn = (rho * vv + 2.0 * w[r] * l[r]) / (rho + 2.0 * w[r]);
        y[r] = y[r] + rho * (v - zn);
        z[r] = zn;
      }
      __syncthreads();
      S.stamp(2);
      admm_it = it;
      if (it % p.check_termination == 0 || it == p.max_iter) {
        S.Cmul(x, Ax);
        S.matvec(S.P, L.ps, x, Px);
        S.CTmul(y, Aty);
        double pr = 0, nAx = 0, nz = 0, spr = 0, snAx = 0, snz = 0;
        double du = 0, nPx = 0, nAty = 0, nq = 0, sdu = 0, snPx = 0, snAty = 0, snq = 0;
        for (int r = tid; r < m; r += kT) {
          const double ie = 1.0 / E[r];
          pr = fmax(pr, fabs((Ax[r] - z[r]) * ie));
          nAx = fmax(nAx, fabs(Ax[r] * ie));
          nz = fmax(nz, fabs(z[r] * ie));
          spr = fmax(spr, fabs(Ax[r] - z[r]));
          snAx = fmax(snAx, fabs(Ax[r]));
          snz = fmax(snz, fabs(z[r]));
        }
        for (int i = tid; i < n; i += kT) {
          const double id = 1.0 / D[i];
          const double rd = Px[i] + q[i] + Aty[i];
          du = fmax(du, fabs(rd * id));
          nPx = fmax(nPx, fabs(Px[i] * id));
          nAty = fmax(nAty, fabs(Aty[i] * id));
          nq = fmax(nq, fabs(q[i] * id));
          sdu = fmax(sdu, fabs(rd));
          snPx = fmax(snPx, fabs(Px[i]));
          snAty = fmax(snAty, fabs(Aty[i]));
          snq = fmax(snq, fabs(q[i]));
        }
        bool nonfinite = false;  // fmax drops NaNs: test the iterate itself
        for (int i = tid; i < n; i += kT) nonfinite = nonfinite || !isfinite(x[i]);
        for (int r = tid; r < m; r += kT) nonfinite = nonfinite || !isfinite(z[r]) || !isfinite(y[r]);
        pr = S.blk.max(pr);
        nAx = S.blk.max(nAx);
        nz = S.blk.max(nz);
        spr = S.blk.max(spr);
        snAx = S.blk.max(snAx);
        snz = S.blk.max(snz);
        du = S.blk.max(du);
        nPx = S.blk.max(nPx);
        nAty = S.blk.max(nAty);
        nq = S.blk.max(nq);
        sdu = S.blk.max(sdu);
        snPx = S.blk.max(snPx);
        snAty = S.blk.max(snAty);
        snq = S.blk.max(snq);
        nonfinite = S.blk.any(nonfinite);
        S.stamp(3);
        const double ic = 1.0 / S.c;
        du *= ic;
        const double ep = p.eps_abs + p.eps_rel * fmax(nAx, nz);
        const double ed = p.eps_abs + p.eps_rel * fmax(fmax(nPx, nAty), nq) * ic;
        if (nonfinite || !isfinite(pr) || !isfinite(du)) {
          bad = true;
          break;
        }
        if (pr <= ep && du <= ed) {
          admm_ok = true;
          break;
        }
        if (it == p.max_iter) {
          approx = pr <= 10.0 * p.eps_abs + 10.0 * p.eps_rel * fmax(nAx, nz) &&
                   du <= 10.0 * p.eps_abs + 10.0 * p.eps_rel * fmax(fmax(nPx, nAty), nq) * ic;
          break;
        }
        const bool near = p.polish_near > 0.0 && it >= 2 * p.check_termination &&
                          fmax(pr / ep, du / ed) < p.polish_near;
        if (p.polish && p.polish_from > 0 && (it >= p.polish_from || near) && it < p.max_iter) {
          for (int i = tid; i < n; i += kT) xp[i] = x[i];
          __syncthreads();
          const int pr_ = wide_polish<FAST>(S, xp, z, p.polish_attempt_max_iter, pol_it, n_fact, n_ls);
          if (pr_ < 0) {
            bad = true;
            break;
          }
          if (pr_ > 0) {
            for (int i = tid; i < n; i += kT) x[i] = xp[i];
            __syncthreads();
            polished = true;
            break;
          }
          refactor = true;
        }
        if (p.adaptive_rho && it % p.adaptive_rho_interval == 0) {
          const double pn = spr / (fmax(snAx, snz) + kDivTol);
          const double dn = sdu / (fmax(fmax(snPx, snAty), snq) + kDivTol);
          double rn = rho * sqrt(pn / (dn + kDivTol));
          rn = fmin(fmax(rn, kRhoMin), kRhoMax);
          if (rn > rho * p.adaptive_rho_tolerance || rn < rho / p.adaptive_rho_tolerance) {
            rho = rn;
            refactor = true;
          }
        }
      }
    }
    st = admm_ok ? MPCQP_SOLVED : (approx ? MPCQP_SOLVED_INACCURATE : MPCQP_MAX_ITER_REACHED);
  }
  const bool do_polish = p.method == MPCQP_METHOD_NEWTON ? true : (p.polish != 0 && admm_ok);
  for (int i = tid; i < n; i += kT) xa[i] = x[i];
  __syncthreads();
  if (polished) {
    st = MPCQP_SOLVED;
  } else if (do_polish && !bad) {
    double* zc = S.at(L.oZc);
    const double* zg = z;
    if (p.method != MPCQP_METHOD_ADMM) {
      S.Cmul(x, zt);  // the C code's zc: C x at the start (x = 0)
      zg = zt;
    }
    (void)zc;
    const int r_ = wide_polish<FAST>(S, x, zg, p.polish_max_iter, pol_it, n_fact, n_ls);
    if (r_ < 0) {
      bad = true;
    } else if (r_ > 0) {
      st = MPCQP_SOLVED;
    } else if (p.method == MPCQP_METHOD_ADMM) {
      for (int i = tid; i < n; i += kT) x[i] = xa[i];
      __syncthreads();
      st = admm_ok ? MPCQP_SOLVED_INACCURATE : MPCQP_MAX_ITER_REACHED;
    } else {
      st = MPCQP_MAX_ITER_REACHED;
    }
  }
  bool nf = false;
  for (int i = tid; i < n; i += kT) nf = nf || !isfinite(x[i]);
  if (S.blk.any(nf)) bad = true;
  if (bad) st = MPCQP_NUMERICAL_ERROR;

  // ---- outputs (unscaled): speeds W -> accelerations, states by the LTV recursion
  const double* mdl = S.at(L.oModel);
  const double* al = mdl;
  const double* be = mdl + N;
  const double* ga = mdl + 2 * N;
  const double* et = mdl + 3 * N;
  const double* si = mdl + 4 * N;
  const double* c0 = mdl + 5 * N;
  const double* c1 = mdl + 6 * N;
  const double* x0 = mdl + 11 * N + 4;
  const double* up = mdl + 11 * N + 8;
  double* Wv = S.at(L.oXt);  // reuse: W
  double* Uv = S.at(L.oRhs);  // reuse: U (interleaved a, delta)
  for (int i = tid; i < n; i += kT) Wv[i] = D[i] * x[i];
  __syncthreads();
  for (int k = tid; k < N; k += kT) {
    Uv[2 * k] = (Wv[2 * k] - (k == 0 ? x0[3] : Wv[2 * k - 2])) / p.dt;
    Uv[2 * k + 1] = Wv[2 * k + 1];
  }
  __syncthreads();
  double* Xb = Xo ? Xo + (size_t)b * 4 * (N + 1) : nullptr;
  if (tid == 0) {
    double X0 = x0[0], X1 = x0[1], X2 = x0[2], X3 = x0[3];
    for (int k = 0; k <= N; ++k) {
      if (Xb) {
        Xb[0 * (N + 1) + k] = X0;
        Xb[1 * (N + 1) + k] = X1;
        Xb[2 * (N + 1) + k] = X2;
        Xb[3 * (N + 1) + k] = X3;
      }
      if (activeo) activeo[(size_t)b * (5 * N + 1) + k] = X3 > p.v_bounds[1] ? 2 : (X3 < p.v_bounds[0] ? 1 : 0);
      if (k == N) break;
      const double psi = X2, v = X3;
      const double nx0 = X0 + al[k] * psi + be[k] * v + c0[k];
      const double nx1 = X1 + ga[k] * psi + et[k] * v + c1[k];
      X2 = psi + si[k] * Uv[2 * k + 1];
      X3 = Wv[2 * k];
      X0 = nx0;
      X1 = nx1;
    }
    statuso[b] = st;
    if (iterso) {
      iterso[4 * (size_t)b + 0] = admm_it;
      iterso[4 * (size_t)b + 1] = pol_it;
      iterso[4 * (size_t)b + 2] = n_fact;
      iterso[4 * (size_t)b + 3] = n_ls;
    }
    if (u0o) {
      u0o[2 * (size_t)b] = Uv[0];
      u0o[2 * (size_t)b + 1] = Uv[1];
    }
  }
  for (int qq = tid; qq < n; qq += kT) {
    const int c = qq & 1, k = qq >> 1;
    if (Uo) Uo[(size_t)b * n + c * N + k] = Uv[qq];
    if (activeo) {
      uint8_t* ab = activeo + (size_t)b * (5 * N + 1);
      const double uu = Uv[qq];
      ab[N + 1 + qq] = uu > p.u_bounds[2 * c + 1] ? 2 : (uu < p.u_bounds[2 * c] ? 1 : 0);
      const double d = uu - (qq < 2 ? up[c] : Uv[qq - 2]);
      ab[3 * N + 1 + qq] = d > p.du_bounds[2 * c + 1] ? 2 : (d < p.du_bounds[2 * c] ? 1 : 0);
    }
  }
}

// kMode: where the arena and Pbar live -- 2 both in LDS, 1 the arena in LDS and Pbar in the
// workspace, 0 both in the workspace.  A compile-time choice, so every access is a ds_* or a
// global_* instruction (a pointer that may be either compiles to flat accesses, which wait for
// all outstanding memory operations: ~100x slower here).
template <int kMode, bool FAST>
__global__ __launch_bounds__(kT) void k_solve_wide(mpcqp_params p, int B, const uint8_t* __restrict__ mask,
                                                   const double* __restrict__ model, double* __restrict__ wide,
                                                   double* __restrict__ u0o, double* __restrict__ Xo,
                                                   double* __restrict__ Uo, int32_t* __restrict__ statuso,
                                                   int32_t* __restrict__ iterso, uint8_t* __restrict__ activeo) {
  extern __shared__ double lds[];
  const int b = blockIdx.x;
  if (b >= B || (mask && !mask[b])) return;
  const int N = p.horizon, n = 2 * N;
  Wide S;
  S.L = WideLayout::make(N);
  S.tid = threadIdx.x;
  S.dt = p.dt;
  S.c = 1.0;
  double* qp = wide + (size_t)b * wide_stride_of(S.L);
  S.in_lds = kMode != 0;
  if constexpr (kMode == 2) {
    S.A = lds;
    S.P = lds + S.L.total;
  } else if constexpr (kMode == 1) {
    S.A = lds;
    S.P = qp;
  } else {
    S.A = qp + (size_t)n * S.L.ps;
    S.P = qp;
  }
  S.blk.red = S.A + S.L.oRed;
  const double* mb = model + (size_t)b * model_stride(N);
  for (int i = S.tid; i < model_stride(N); i += kT) S.A[S.L.oModel + i] = mb[i];
  __syncthreads();
#ifdef MPCQP_WIDE_STAMPS
  if constexpr (kMode != 0) {
    S.st = qp + (size_t)n * S.L.ps;
    if (S.tid < 16) S.st[S.tid] = 0.0;
    __syncthreads();
  }
#endif
  S.mark();
  const bool bad = wide_setup(p, S);
  S.stamp(0);
  wide_solve<FAST>(p, S, bad, b, u0o, Xo, Uo, statuso, iterso, activeo);
}

}  // namespace

namespace mpcqp {
size_t wide_stride(int horizon) { return wide_stride_of(WideLayout::make(horizon)); }

void launch_solve_wide(hipStream_t s, const Launch& L) {
  double* wide = L.state;
  const WideLayout lay = WideLayout::make(L.p->horizon);
  const size_t arena = sizeof(double) * (size_t)lay.total, pbar = sizeof(double) * (size_t)lay.n * lay.ps;
  constexpr size_t kLds = 160u * 1024u;
  auto go = [&](auto kern, size_t lds) {
    if (lds > 65536)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
    hipLaunchKernelGGL(kern, dim3(L.B), dim3(kT), lds, s, *L.p, L.B, L.mask, L.model, wide, L.u0, L.X, L.U, L.st,
                       L.it, L.ac);
  };
  // reproducible = 1: the C restatement op for op; 0 (N >= MPCQP_WIDE_MIN_HORIZON): the fast polish
  const bool fast = L.p->reproducible == 0;
  if (arena + pbar <= kLds)
    fast ? go(&k_solve_wide<2, true>, arena + pbar) : go(&k_solve_wide<2, false>, arena + pbar);
  else if (arena <= kLds)
    fast ? go(&k_solve_wide<1, true>, arena) : go(&k_solve_wide<1, false>, arena);
  else
    fast ? go(&k_solve_wide<0, true>, 0) : go(&k_solve_wide<0, false>, 0);
}
}  // namespace mpcqp
