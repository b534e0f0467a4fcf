// Small elementwise kernels of the fused step (gfx950).
//
// center_rows_kernel: the centred per-model input of threshold / learned-centre SAEs,
//   out[g, b, :] = bf16(x[b, :] - c[g, :]),  x bf16 [B, d] shared, c fp32 [G, d]
// in one pass (the torch form was an fp32 [G, B, d] subtraction plus a bf16 copy).
// gather_rows_kernel: the step's batch fetch from the HBM activation ring, out[i] = buf[idx[i]]
//   for 16-byte-multiple rows: one wave per row, every lane one dwordx4 per 1 KiB of the row
//   (the torch index_select took 5.3 us for 2048 x 1 KiB rows, mostly its launch tail).
#include "common.h"

namespace scamd {

__global__ __launch_bounds__(256) void center_rows_kernel(const uint16_t* __restrict__ x, const float* __restrict__ c,
                                                          uint16_t* __restrict__ out, int G, int B, int d) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;  // one thread per 4 elements of out
  const long per_model = (long)B * d / 4;
  if (t >= (long)G * per_model) return;
  const int g = (int)(t / per_model);
  const long e = (t - (long)g * per_model) * 4;  // element offset inside [B, d]
  const int k = (int)(e % d);
  const ushort4 xv = *reinterpret_cast<const ushort4*>(x + e);
  const float4 cv = *reinterpret_cast<const float4*>(c + (long)g * d + k);
  *reinterpret_cast<ushort4*>(out + (long)g * B * d + e) =
      make_ushort4(f2bf(bf2f(xv.x) - cv.x), f2bf(bf2f(xv.y) - cv.y), f2bf(bf2f(xv.z) - cv.z), f2bf(bf2f(xv.w) - cv.w));
}

__global__ __launch_bounds__(256) void gather_rows_kernel(const u32x4_t* __restrict__ buf, const long* __restrict__ idx,
                                                          u32x4_t* __restrict__ out, long rows, int row_vec) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63;
  const long src = idx[r];
  const u32x4_t* s = buf + src * row_vec;
  u32x4_t* o = out + r * row_vec;
  for (int v = lane; v < row_vec; v += 64) o[v] = s[v];
}

}  // namespace scamd

using namespace scamd;

extern "C" {

int sc_center_rows(const void* x, const float* c, void* out, int G, int B, int d, hipStream_t stream) {
  if (d % 4 || G < 1 || B < 1) return 1;
  const long total = (long)G * B * d / 4;
  hipLaunchKernelGGL(center_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream,
                     reinterpret_cast<const uint16_t*>(x), c, reinterpret_cast<uint16_t*>(out), G, B, d);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int sc_gather_rows(const void* buf, const long* idx, void* out, long rows, long row_bytes, hipStream_t stream) {
  if (row_bytes % 16 || rows < 0) return 1;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream,
                     reinterpret_cast<const u32x4_t*>(buf), idx, reinterpret_cast<u32x4_t*>(out), rows,
                     (int)(row_bytes / 16));
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
