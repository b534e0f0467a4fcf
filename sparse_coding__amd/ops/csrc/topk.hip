// Top-k sparse coding kernels for an ensemble with per-model k (gfx950).
//
// Reference: TopKEncoder (autoencoders/topk_encoder.py:19-40): scores = x D^T,
// keep each row's top-k, ReLU, x_hat = code D, MSE.  The reference cannot
// vmap over models because k changes the output shape (no_stacking=True,
// big_sweep_experiments.py:246-253); here k lives in device memory and every
// model runs in the same launches:
//   topk_select_kernel   : exact per-row radix select (4 x 8-bit passes over the
//                          orderable bit pattern, LDS histograms), scores kept in
//                          registers; emits (idx, value) pairs.
//   topk_decode_grad     : one wave per row: sparse decode x_hat = sum_j v_j D[idx_j]
//                          (bf16 dictionary gathered from L2), residual, per-row
//                          squared error, then the k code gradients <R, D[idx_j]>
//                          scattered into dense bf16 buffers for the MFMA wgrad GEMM.
//   topk_clear           : zeroes exactly the scattered positions afterwards.
#include "common.h"

namespace scamd {

__device__ __forceinline__ uint32_t order_key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // larger float -> larger key
}

template <int PER>  // keys per thread (n <= 256 * PER)
__global__ __launch_bounds__(256) void topk_select_kernel(const float* __restrict__ scores, const int* __restrict__ kv,
                                                          int* __restrict__ idx, float* __restrict__ val, int B, int n,
                                                          int kmax, int absolute, int relu) {
  __shared__ uint32_t hist[256];
  __shared__ int sel[4];  // digit, count above, out cursor, tie cursor
  const long row = blockIdx.x;
  const int g = row / B;
  const int k = min(kv[g], n);
  const float* S = scores + row * n;
  const int tid = threadIdx.x;
  uint32_t key[PER];
  float sv[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = tid + i * 256;
    const float s = c < n ? S[c] : 0.f;
    sv[i] = s;
    key[i] = c < n ? order_key(absolute ? fabsf(s) : s) : 0u;  // padding sorts below every real key
  }
  uint32_t prefix = 0, mask = 0;
  int remaining = k;
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if (tid + i * 256 < n && (key[i] & mask) == prefix) atomicAdd(&hist[(key[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      int above = 0, b = 255;
      for (; b > 0; --b) {
        if (above + (int)hist[b] >= remaining) break;
        above += hist[b];
      }
      sel[0] = b;
      sel[1] = above;
    }
    __syncthreads();
    prefix |= (uint32_t)sel[0] << shift;
    mask |= 255u << shift;
    remaining -= sel[1];
    __syncthreads();
  }
  // prefix is now the k-th largest key; take everything above it and `remaining` ties
  if (tid == 0) { sel[2] = 0; sel[3] = 0; }
  __syncthreads();
  int* I = idx + row * kmax;
  float* V = val + row * kmax;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = tid + i * 256;
    if (c >= n || k == 0) continue;
    bool take = key[i] > prefix;
    if (!take && key[i] == prefix) take = atomicAdd(&sel[3], 1) < remaining;
    if (take) {
      const int pos = atomicAdd(&sel[2], 1);
      I[pos] = c;
      V[pos] = relu ? fmaxf(sv[i], 0.f) : sv[i];
    }
  }
  // pad the unused slots of models with k < kmax
  for (int j = k + tid; j < kmax; j += 256) {
    I[j] = 0;
    V[j] = 0.f;
  }
}

// One wave per (model, row).  D: [G][n][d] bf16 normalised dictionary (gathered rows).
template <int NV>  // d == 256 * NV ... handled generically with NV = ceil(d / 256)
__global__ __launch_bounds__(256) void topk_decode_grad_kernel(
    const int* __restrict__ idx, const float* __restrict__ val, const int* __restrict__ kv,
    const uint16_t* __restrict__ D, const uint16_t* __restrict__ X, long sx, uint16_t* __restrict__ R,
    float* __restrict__ row_se, uint16_t* __restrict__ codebuf, uint16_t* __restrict__ dscbuf, int G, int B,
    int n, int d, int kmax) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)G * B) return;
  const int g = row / B, b = row % B;
  const int k = min(kv[g], kmax);
  const int* I = idx + row * kmax;
  const float* V = val + row * kmax;
  const uint16_t* Dg = D + (long)g * n * d;
  float acc[NV * 4];
#pragma unroll
  for (int e = 0; e < NV * 4; ++e) acc[e] = 0.f;
  for (int j = 0; j < k; ++j) {
    const float w = V[j];
    if (w == 0.f) continue;  // wave-uniform
    const uint16_t* Dr = Dg + (long)I[j] * d;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int e = (v * 64 + lane) * 4;
      if (e < d) {
        const ushort4 h = *reinterpret_cast<const ushort4*>(Dr + e);
        acc[v * 4 + 0] += w * bf2f(h.x);
        acc[v * 4 + 1] += w * bf2f(h.y);
        acc[v * 4 + 2] += w * bf2f(h.z);
        acc[v * 4 + 3] += w * bf2f(h.w);
      }
    }
  }
  // residual R = x_hat - x (kept in fp32 registers for the code gradients)
  const uint16_t* Xr = X + (long)g * sx + (long)b * d;
  uint16_t* Rr = R + row * d;
  float se = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int e = (v * 64 + lane) * 4;
    if (e < d) {
      const ushort4 h = *reinterpret_cast<const ushort4*>(Xr + e);
      acc[v * 4 + 0] -= bf2f(h.x);
      acc[v * 4 + 1] -= bf2f(h.y);
      acc[v * 4 + 2] -= bf2f(h.z);
      acc[v * 4 + 3] -= bf2f(h.w);
      se += acc[v * 4 + 0] * acc[v * 4 + 0] + acc[v * 4 + 1] * acc[v * 4 + 1] +
            acc[v * 4 + 2] * acc[v * 4 + 2] + acc[v * 4 + 3] * acc[v * 4 + 3];
      *reinterpret_cast<ushort4*>(Rr + e) =
          make_ushort4(f2bf(acc[v * 4 + 0]), f2bf(acc[v * 4 + 1]), f2bf(acc[v * 4 + 2]), f2bf(acc[v * 4 + 3]));
    }
  }
  se = wave_sum(se);
  if (lane == 0) row_se[row] = se;
  if (!codebuf) return;
  // code gradients (units of R): dscore_j = 1[v_j > 0] <R, D[idx_j]>; scatter code and dscore
  uint16_t* Cb = codebuf + row * (long)n;
  uint16_t* Sb = dscbuf + row * (long)n;
  for (int j = 0; j < k; ++j) {
    const float w = V[j];
    const uint16_t* Dr = Dg + (long)I[j] * d;
    float dot = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int e = (v * 64 + lane) * 4;
      if (e < d) {
        const ushort4 h = *reinterpret_cast<const ushort4*>(Dr + e);
        dot += acc[v * 4 + 0] * bf2f(h.x) + acc[v * 4 + 1] * bf2f(h.y) + acc[v * 4 + 2] * bf2f(h.z) +
               acc[v * 4 + 3] * bf2f(h.w);
      }
    }
    dot = wave_sum(dot);
    if (lane == 0 && w > 0.f) {
      Cb[I[j]] = f2bf(w);
      Sb[I[j]] = f2bf(dot);
    }
  }
}

__global__ __launch_bounds__(256) void topk_clear_kernel(const int* __restrict__ idx, uint16_t* __restrict__ a,
                                                         uint16_t* __restrict__ b, long rows, int n, int kmax) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= rows * kmax) return;
  const long row = t / kmax;
  const int c = idx[t];
  a[row * n + c] = 0;
  b[row * n + c] = 0;
}

}  // namespace scamd

using namespace scamd;

extern "C" {

int sc_topk_select(const float* scores, const int* k, int* idx, float* val, int G, int B, int n, int kmax,
                   int absolute, int relu, hipStream_t stream) {
  const int per = (n + 255) / 256;
  dim3 grid((unsigned)G * B);
#define SC_T(P) \
  if (per <= P) { hipLaunchKernelGGL((topk_select_kernel<P>), grid, dim3(256), 0, stream, scores, k, idx, val, B, n, kmax, absolute, relu); \
    return hipGetLastError() == hipSuccess ? 0 : 3; }
  SC_T(4) SC_T(8) SC_T(16) SC_T(32) SC_T(64)
#undef SC_T
  return 1;
}

int sc_topk_decode_grad(const int* idx, const float* val, const int* k, const void* D, const void* X, long sx,
                        void* R, float* row_se, void* codebuf, void* dscbuf, int G, int B, int n, int d, int kmax,
                        hipStream_t stream) {
  if (d % 4) return 1;
  const int nv = (d + 255) / 256;
  dim3 grid(((long)G * B + 3) / 4);
#define SC_D(V) \
  if (nv <= V) { hipLaunchKernelGGL((topk_decode_grad_kernel<V>), grid, dim3(256), 0, stream, idx, val, k, \
      reinterpret_cast<const uint16_t*>(D), reinterpret_cast<const uint16_t*>(X), sx, reinterpret_cast<uint16_t*>(R), \
      row_se, reinterpret_cast<uint16_t*>(codebuf), reinterpret_cast<uint16_t*>(dscbuf), G, B, n, d, kmax); \
    return hipGetLastError() == hipSuccess ? 0 : 3; }
  SC_D(1) SC_D(2) SC_D(3) SC_D(4) SC_D(8) SC_D(16)
#undef SC_D
  return 1;
}

int sc_topk_clear(const int* idx, void* a, void* b, long rows, int n, int kmax, hipStream_t stream) {
  const long total = rows * kmax;
  hipLaunchKernelGGL(topk_clear_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, idx,
                     reinterpret_cast<uint16_t*>(a), reinterpret_cast<uint16_t*>(b), rows, n, kmax);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
