// Synthetic sparse-code generation (gfx950): the sampling half of the reference's
// generate_rand_dataset / generate_correlated_dataset (reference sc_datasets/random_dataset.py:
// 160-188, :191-245) as one elementwise kernel with a counter-based RNG, so the codes are
// produced directly in bf16 for the MFMA GEMM that mixes them into activations
// (x = codes @ feats; ops/gemm.matmul_nn, output straight into the HBM ring).
//
//   code[b, j] = (u1 <= p[j]) ? u2 * u3 : 0        u1, u2, u3 ~ U[0, 1) from Philox4x32-10
//
// Philox is keyed by (seed) and countered by (row, column, stream offset): any slice of any
// batch is reproducible independently of launch geometry.
#include "common.h"

namespace scamd {

__device__ __forceinline__ void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                             uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
  const uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
  const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
  c0 = n0;
  c1 = lo1;
  c2 = n2;
  c3 = lo0;
}

__device__ __forceinline__ void philox4x32_10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                              uint32_t k1) {
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c0, c1, c2, c3, k0, k1);
    k0 += W0;
    k1 += W1;
  }
}

__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }  // [0, 1)

// One thread per 4 consecutive columns of one row (one Philox call per element, 3 of its 4
// words used).  probs: [n] fp32; out: [B, n] bf16 (n % 4 == 0).
__global__ __launch_bounds__(256) void synth_codes_kernel(const float* __restrict__ probs, uint16_t* __restrict__ out,
                                                          long B, int n, uint32_t seed_lo, uint32_t seed_hi,
                                                          unsigned long long row0) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  const long per_row = n / 4;
  if (t >= B * per_row) return;
  const long b = t / per_row;
  const int j0 = (int)(t - b * per_row) * 4;
  const unsigned long long row = row0 + (unsigned long long)b;
  ushort4 o;
  uint16_t* op = reinterpret_cast<uint16_t*>(&o);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t c0 = (uint32_t)row, c1 = (uint32_t)(row >> 32), c2 = (uint32_t)(j0 + q), c3 = 0x5C0DE5u;
    philox4x32_10(c0, c1, c2, c3, seed_lo, seed_hi);
    const float v = u01(c0) <= probs[j0 + q] ? u01(c1) * u01(c2) : 0.f;
    op[q] = f2bf(v);
  }
  *reinterpret_cast<ushort4*>(out + b * (long)n + j0) = o;
}

}  // namespace scamd

using namespace scamd;

extern "C" {

// codes [B, n] bf16 for rows row0 .. row0 + B - 1 of the (seed) stream.
int sc_synth_codes(const float* probs, void* out, long B, int n, unsigned long long seed, unsigned long long row0,
                   hipStream_t stream) {
  if (n % 4 || B < 1) return 1;
  const long total = B * (n / 4);
  hipLaunchKernelGGL(synth_codes_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, probs,
                     reinterpret_cast<uint16_t*>(out), B, n, (uint32_t)seed, (uint32_t)(seed >> 32), row0);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
