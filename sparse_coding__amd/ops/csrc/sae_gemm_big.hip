// 256x256 block instantiations of the grouped SAE GEMM (see sae_gemm_kernel.h; 256x128 blocks:
// sae_gemm_256x128.hip).  Built WITHOUT -amdgpu-mfma-vgpr-form: these shapes keep 128
// accumulator registers per wave in AGPRs.
#include "sae_gemm_kernel.h"

namespace scamd {

int launch_big(int shape, int pipe, int epi, bool ak, bool bk, const GemmParams& p, int nprob, hipStream_t stream) {
  // (256x256 as sixteen 64x64 waves on BK32 x 3, one block of 16 waves per CU, measured no faster for the
  // weight gradients and slower for the top-k GEMMs: profiles/r6/w16/, scripts/lab/w16_256x256_r6.patch)
  if (shape == 3) {
    if (pipe == 1) return launch<S256, 32, 4, false>(epi, ak, bk, p, nprob, stream);
    if (pipe == 3) return launch<S256, 32, 3, false>(epi, ak, bk, p, nprob, stream);
    if (pipe == 2) return launch<S256, 32, 2, false>(epi, ak, bk, p, nprob, stream);
    return launch<S256, 64, 2>(epi, ak, bk, p, nprob, stream);
  }
  return launch_256x128(pipe, epi, ak, bk, p, nprob, stream);
}

}  // namespace scamd
