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

}  // extern "C"
