// 256x256 block instantiations of the grouped SAE GEMM (see sae_gemm_kernel.h; 256x128 blocks:
// sae_gemm_256x128.hip).  Built WITHOUT -amdgpu-mfma-vgpr-form: these shapes keep 128
// accumulator registers per wave in AGPRs.
#include "sae_gemm_kernel.h"

namespace scamd {

int launch_big(int shape, int pipe, int epi, bool ak, bool bk, const GemmParams& p, int nprob, hipStream_t stream,
               bool w16) {
  // (lab) 256x256 as SIXTEEN 64x64 waves on BK32 x 3 (96 KB, one block of 16 waves per CU)
  if (shape == 3 && w16 && pipe == 3) return launch<Shape<4, 4, 4, 4>, 32, 3, false>(epi, ak, bk, p, nprob, stream);
  if (shape == 3) {
    if (pipe == 1) return launch<S256, 32, 4, false>(epi, ak, bk, p, nprob, stream);
    if (pipe == 3) return launch<S256, 32, 3, false>(epi, ak, bk, p, nprob, stream);
    if (pipe == 2) return launch<S256, 32, 2, false>(epi, ak, bk, p, nprob, stream);
    return launch<S256, 64, 2>(epi, ak, bk, p, nprob, stream);
  }
  return launch_256x128(pipe, epi, ak, bk, p, nprob, stream);
}

}  // namespace scamd
