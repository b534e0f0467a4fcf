// Shared CDNA4 (gfx950) helpers for the sparse-coding kernels.
//
// Everything here is wave64 / MFMA specific: this code is written for MI355X
// only (hipcc --offload-arch=gfx950) and has no other target.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace scamd {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef short i16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

#define SC_LDS(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ float bf2f(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}

// Round-to-nearest-even f32 -> bf16 (hipcc lowers the cast to v_cvt_pk_bf16_f32,
// which keeps NaN a NaN).
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

// DPP lane shuffle of a float (row_shr / row_bcast controls; lanes whose source is outside
// the row read 0, so adding the result is a scan step).
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xf, false));
}

// Inclusive scan within each 16-lane row: lane 15 of a row ends with the row's sum.
__device__ __forceinline__ float row16_scan(float v) {
  v += dpp_f<0x111>(v);  // row_shr:1
  v += dpp_f<0x112>(v);  // row_shr:2
  v += dpp_f<0x114>(v);  // row_shr:4
  v += dpp_f<0x118>(v);  // row_shr:8
  return v;
}

// Wave-wide sum on the DPP path (row scans, row broadcasts, lane 63 read back): six VALU
// adds and a readlane instead of six ds_bpermute round trips.  Uniform result.
__device__ __forceinline__ float wave_sum(float v) {
  v = row16_scan(v);
  v += dpp_f<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
  v += dpp_f<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for a 256-thread block; `red` must hold >= 4 floats of LDS.
__device__ __forceinline__ float block_sum_256(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return r;
}

// Block-wide sum over NW waves; `red` must hold >= NW floats of LDS.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) r += red[i];
  __syncthreads();
  return r;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops, not for its
// global stores / loads / LDS-DMAs (a __syncthreads() would drain vmcnt too).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// block_sum with LDS-only barriers (see lds_barrier); `red` must hold >= NW floats.
template <int NW>
__device__ __forceinline__ float block_sum_lds(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  lds_barrier();
  if (lane == 0) red[w] = v;
  lds_barrier();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) r += red[i];
  lds_barrier();
  return r;
}

// Two block-wide sums behind ONE LDS-only barrier, for a block's last reduction: `red` (>= 2 NW
// floats) is not reused afterwards, so the barrier that protects a reused scratch is not needed.
// Every thread gets both totals (same summation order as block_sum_lds: bit-identical).
template <int NW>
__device__ __forceinline__ float2 block_sum2_final(float a, float b, float* red) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red[2 * w] = a;
    red[2 * w + 1] = b;
  }
  lds_barrier();
  float2 r = make_float2(0.f, 0.f);
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    r.x += red[2 * i];
    r.y += red[2 * i + 1];
  }
  return r;
}

// Bijective XCD-aware block remap (MI355X has 8 XCDs, each with its own L2).
// Hardware hands consecutive block ids to different XCDs round-robin; this
// gives each XCD a contiguous run of logical tiles so neighbouring tiles that
// share operand panels hit the same L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

}  // namespace scamd
