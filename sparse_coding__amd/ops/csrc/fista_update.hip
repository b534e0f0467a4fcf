// FISTA dictionary-learning update on the device (gfx950): the Hessian-diagonal EMA and the
// quadratic basis update of the fork's iterative dictionary learning (reference
// autoencoders/fista.py:88-96 and :131-138), for every model of an ensemble in one launch.
//
//   hessian_ema_kernel : H <- keep * H + scale * sum_b A[b, j]^2           (per model, per atom)
//   basis_apply_kernel : D[j, :] += dBt[j, :] / (H[j] + lowest)  (dBt = step/B * A^T Res, from
//                        the grouped MFMA GEMM), optional clamp at 0, then renormalise -- per
//                        atom (rows, the intended unit-norm dictionary) or per activation
//                        dimension (columns, the reference's D.norm(2, 0), SURVEY B#4); also
//                        writes the bf16 copy the next FISTA solve multiplies by.
// Both are bandwidth-trivial next to the 300-iteration solve; they exist so the whole update
// stays on the GPU with no fp32 torch bmm / elementwise chain in between.
#include "common.h"

namespace scamd {

// One block per (model, 64-column strip): thread (rg, c) sums rows rg, rg+4, ... of column c,
// then the four row-group partials are added in LDS (fixed order: deterministic).
__global__ __launch_bounds__(256) void hessian_ema_kernel(const float* __restrict__ A, float* __restrict__ H, int B,
                                                          int n, float keep, float scale) {
  __shared__ float part[4][64];
  const int g = blockIdx.y, c0 = blockIdx.x * 64;
  const int c = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const float* Ag = A + (long)g * B * n + c0 + c;
  float s = 0.f;
#pragma unroll 8
  for (int b = rg; b < B; b += 4) {
    const float v = Ag[(long)b * n];
    s += v * v;
  }
  part[rg][c] = s;
  __syncthreads();
  if (rg == 0) {
    const float t = part[0][c] + part[1][c] + part[2][c] + part[3][c];
    float* h = H + (long)g * n + c0 + c;
    *h = keep * *h + scale * t;
  }
}

// Row mode: one wave per atom row (d <= 64 * 64 handled by the lane loop).
__global__ __launch_bounds__(256) void basis_apply_rows_kernel(float* __restrict__ D, const float* __restrict__ dBt,
                                                               const float* __restrict__ H, uint16_t* __restrict__ Db,
                                                               long rows, int n, int d, float lowest, int nonneg) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const float inv = 1.f / (H[row] + lowest);  // H is [G, n] = one entry per row of [G * n, d]
  float* Dr = D + row * d;
  const float* Ur = dBt + row * d;
  float ss = 0.f;
  for (int k = lane; k < d; k += 64) {
    float v = Dr[k] + Ur[k] * inv;
    if (nonneg) v = fmaxf(v, 0.f);
    Dr[k] = v;
    ss += v * v;
  }
  const float r = 1.f / fmaxf(sqrtf(wave_sum(ss)), 1e-8f);
  for (int k = lane; k < d; k += 64) {
    const float v = Dr[k] * r;
    Dr[k] = v;
    if (Db) Db[row * d + k] = f2bf(v);
  }
}

// Column mode: one block per (model, 64-column strip): pass 1 updates every atom's 64 entries
// and sums their squares per column (four row groups, LDS reduction), pass 2 rescales.
__global__ __launch_bounds__(256) void basis_apply_cols_kernel(float* __restrict__ D, const float* __restrict__ dBt,
                                                               const float* __restrict__ H, uint16_t* __restrict__ Db,
                                                               int n, int d, float lowest, int nonneg) {
  __shared__ float part[4][64];
  const int g = blockIdx.y, c0 = blockIdx.x * 64;
  const int c = threadIdx.x & 63, rg = threadIdx.x >> 6;
  float* Dg = D + (long)g * n * d + c0 + c;
  const float* Ug = dBt + (long)g * n * d + c0 + c;
  const float* Hg = H + (long)g * n;
  float s = 0.f;
  for (int j = rg; j < n; j += 4) {
    float v = Dg[(long)j * d] + Ug[(long)j * d] / (Hg[j] + lowest);
    if (nonneg) v = fmaxf(v, 0.f);
    Dg[(long)j * d] = v;
    s += v * v;
  }
  part[rg][c] = s;
  __syncthreads();
  const float r = 1.f / fmaxf(sqrtf(part[0][c] + part[1][c] + part[2][c] + part[3][c]), 1e-30f);
  for (int j = rg; j < n; j += 4) {
    const float v = Dg[(long)j * d] * r;
    Dg[(long)j * d] = v;
    if (Db) Db[(long)g * n * d + (long)j * d + c0 + c] = f2bf(v);
  }
}

// Adjoint of the unrolled FISTA loop (the "FISTA in the loss" objective, reference
// autoencoders/fista.py:141-172), one elementwise pass per iteration t = T-1 .. 0 over
// [G][B][n].  Forward: V_t = Y_t + eta (X - Y_t D) D^T, A_{t+1} = relu(V_t - eta lam),
// Y_{t+1} = A_{t+1} + m_t (A_{t+1} - A_t), Y_0 = A_0 = c.  With nS = -(Vbar_t D) (GEMM) and
// T2 = nS D^T (GEMM):
//   Ybar_t = Vbar_t + eta T2
//   t >= 1: Abar_t = (1 + m_{t-1}) Ybar_t - m_t Ybar_{t+1};  Vbar_{t-1} = Abar_t 1[A_t > 0]
//   t == 0: cbar = Ybar_0 - m_0 Ybar_1
// Slab slot s of Asave holds A_{s+1}; Vbar_{t-1} also goes to slab slot t-1 (bf16) for the
// dictionary-gradient GEMM.
__global__ __launch_bounds__(256) void fista_adjoint_kernel(const float* __restrict__ T2, float* __restrict__ Vbar,
                                                            const float* __restrict__ Ynext, float* __restrict__ Ycur,
                                                            const uint16_t* __restrict__ Aslab,
                                                            uint16_t* __restrict__ Vslab, float* __restrict__ cbar,
                                                            const float* __restrict__ eta, float m_prev, float m_t,
                                                            int B, int n, int T, int t, long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const long per = (long)B * n;
  const int g = (int)(i / per);
  const long e = i - (long)g * per;
  const float yb = Vbar[i] + eta[g] * T2[i];
  const float yn = Ynext[i];
  Ycur[i] = yb;
  if (t == 0) {
    cbar[i] = yb - m_t * yn;
    return;
  }
  const long slot = ((long)g * T + (t - 1)) * per + e;  // A_t lives in slot t - 1
  const float ab = (1.f + m_prev) * yb - m_t * yn;
  const float v = bf2f(Aslab[slot]) > 0.f ? ab : 0.f;
  Vbar[i] = v;
  Vslab[slot] = f2bf(v);
}

// Start of the sweep: Vbar_{T-1} = -(Rbar D^T) 1[A_T > 0] (T2 = Rbar D^T from the GEMM).
__global__ __launch_bounds__(256) void fista_adjoint_init_kernel(const float* __restrict__ T2, float* __restrict__ Vbar,
                                                                 const uint16_t* __restrict__ Aslab,
                                                                 uint16_t* __restrict__ Vslab, int B, int n, int T,
                                                                 long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const long per = (long)B * n;
  const int g = (int)(i / per);
  const long slot = ((long)g * T + (T - 1)) * per + (i - (long)g * per);
  const float v = bf2f(Aslab[slot]) > 0.f ? -T2[i] : 0.f;
  Vbar[i] = v;
  Vslab[slot] = f2bf(v);
}

}  // namespace scamd

using namespace scamd;

extern "C" {

// H [G, n] <- H * (history - 1) / history + mean_b(A^2) / history, A [G, B, n] fp32.
int sc_hessian_ema(const float* A, float* H, int G, int B, int n, float history, hipStream_t stream) {
  if (n % 64 || G < 1 || B < 1 || history <= 0.f) return 1;
  hipLaunchKernelGGL(hessian_ema_kernel, dim3(n / 64, G), dim3(256), 0, stream, A, H, B, n,
                     (history - 1.f) / history, 1.f / (history * (float)B));
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// D [G, n, d] += dBt / (H + lowest) (per atom), optional clamp, renormalise rows (mode 1) or
// columns (mode 0); Db (optional) receives the bf16 copy.
int sc_basis_apply(float* D, const float* dBt, const float* H, void* Db, int G, int n, int d, float lowest,
                   int nonneg, int mode, hipStream_t stream) {
  if (G < 1 || n < 1 || d < 1) return 1;
  uint16_t* db = reinterpret_cast<uint16_t*>(Db);
  if (mode == 1) {
    const long rows = (long)G * n;
    hipLaunchKernelGGL(basis_apply_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream, D, dBt, H, db,
                       rows, n, d, lowest, nonneg);
  } else {
    if (d % 64) return 1;
    hipLaunchKernelGGL(basis_apply_cols_kernel, dim3(d / 64, G), dim3(256), 0, stream, D, dBt, H, db, n, d, lowest,
                       nonneg);
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int sc_fista_adjoint(const float* T2, float* Vbar, const float* Ynext, float* Ycur, const void* Aslab, void* Vslab,
                     float* cbar, const float* eta, float m_prev, float m_t, int G, int B, int n, int T, int t,
                     hipStream_t stream) {
  if (t < 0 || t >= T || (t == 0 && !cbar)) return 1;
  const long total = (long)G * B * n;
  hipLaunchKernelGGL(fista_adjoint_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, T2, Vbar,
                     Ynext, Ycur, reinterpret_cast<const uint16_t*>(Aslab), reinterpret_cast<uint16_t*>(Vslab), cbar,
                     eta, m_prev, m_t, B, n, T, t, total);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int sc_fista_adjoint_init(const float* T2, float* Vbar, const void* Aslab, void* Vslab, int G, int B, int n, int T,
                          hipStream_t stream) {
  if (T < 1) return 1;
  const long total = (long)G * B * n;
  hipLaunchKernelGGL(fista_adjoint_init_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, T2,
                     Vbar, reinterpret_cast<const uint16_t*>(Aslab), reinterpret_cast<uint16_t*>(Vslab), B, n, T,
                     total);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
