// 256x128 and 256x256 block instantiations of the grouped SAE GEMM (see
// sae_gemm_kernel.h).  Built WITHOUT -amdgpu-mfma-vgpr-form: these shapes keep 128
// accumulator registers per wave in AGPRs.
#include "sae_gemm_kernel.h"

namespace scamd {

int launch_big(int shape, int pipe, int epi, bool ak, bool bk, const GemmParams& p, int nprob, hipStream_t stream) {
  if (shape == 3) {
    if (pipe == 1) return launch<S256, 32, 4, false>(epi, ak, bk, p, nprob, stream);
    if (pipe == 3) return launch<S256, 32, 3, false>(epi, ak, bk, p, nprob, stream);
    if (pipe == 2) return launch<S256, 32, 2, false>(epi, ak, bk, p, nprob, stream);
    return launch<S256, 64, 2>(epi, ak, bk, p, nprob, stream);
  }
  // 256x128 with the BK32 rings: 72 KB (3 stages) / 48 KB (2 stages) of LDS -> 2 / 3 blocks per CU;
  // the step's K = 512 GEMMs then launch G B n / 32768 blocks (1024 at the headline: 2 full rounds)
  if (pipe == 3) return launch<S256x128, 32, 3, false>(epi, ak, bk, p, nprob, stream);
  if (pipe == 2) return launch<S256x128, 32, 2, false>(epi, ak, bk, p, nprob, stream);
  if (pipe) return 8;
  return launch<S256x128, 64, 2>(epi, ak, bk, p, nprob, stream);
}

}  // namespace scamd
