// 256x128 block instantiations of the grouped SAE GEMM (see sae_gemm_kernel.h): four waves of 128x64,
// one block per CU at the BK64 x 2 ring, with the software-pipelined K loop.  Built WITH
// -amdgpu-mfma-vgpr-form (build.py): in the AGPR form the pipelined loop's two MFMA groups made the
// register allocator copy the 128 accumulators through v_accvgpr moves every iteration; in the VGPR
// form they fit the 256 architectural registers with the two fragment sets (no scratch).
#include "sae_gemm_kernel.h"

namespace scamd {

int launch_256x128(int pipe, int epi, bool ak, bool bk, const GemmParams& p, int nprob, hipStream_t stream) {
  // (256x128 on the BK32 rings, two blocks per CU, measured slower in the step: 0.302-0.307 vs
  // 0.296-0.297 ms, profiles/r5/batch3/cfg14.jsonl)
  // pipe 3: EIGHT waves of 64x64 on the BK32 x 3 ring (72 KB, <= 128 VGPRs: two blocks per CU) -- the
  // encoder / masked code gradient default (ops/gemm.py _CFG_DEFAULT, profiles/r6/w8/)
  if (pipe == 3) return launch<S256x128w8, 32, 3, false>(epi, ak, bk, p, nprob, stream);
  if (pipe) return 8;
  return launch<S256x128, 64, 2>(epi, ak, bk, p, nprob, stream);
}

}  // namespace scamd
