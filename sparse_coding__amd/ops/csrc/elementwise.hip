// Small elementwise kernels of the fused step (gfx950).
//
// center_rows_kernel: the centred per-model input of threshold / learned-centre SAEs,
//   out[g, b, :] = bf16(x[b, :] - c[g, :]),  x bf16 [B, d] shared, c fp32 [G, d]
// in one pass (the torch form was an fp32 [G, B, d] subtraction plus a bf16 copy).
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

}  // extern "C"
