// Grouped bf16 MFMA GEMM with fused sparse-autoencoder epilogues (gfx950): C ABI and the
// 128x128-block launches.  The kernel itself and the epilogue catalogue are in
// sae_gemm_kernel.h; the 256-row block shapes are instantiated in sae_gemm_big.hip.
#include "sae_gemm_kernel.h"


using namespace scamd;

// ------------------------------------------------------------------ C ABI
extern "C" {

struct ScOperand {
  const void* ptr;
  long ld, sg;
};


// Block shape chosen by sc_gemm when cfg == 0: the largest tile that divides the problem,
// gives at least one block per CU (256 CUs on MI355X) and does not end on a mostly idle last
// wave of blocks -- 256x256 runs one block per CU, 128x128 two: the larger tile must fill
// its waves at least as well (within 10 %) as 128x128 would.  (Top-k weight gradient,
// 576 blocks of 256x256 = 2.25 waves: 128x128 measured 1.165 vs 1.201 ms/step.)
static double wave_fill(long blocks, long slots) { return (double)blocks / (double)(slots * ((blocks + slots - 1) / slots)); }
int sc_gemm_shape(int M, int N, int G, int nprob) {
  if (fits<S256>(M, N) && n_blocks<S256>(M, N, G, nprob) >= 256) {
    const double f128 = wave_fill(n_blocks<S128>(M, N, G, nprob), 512);
    return wave_fill(n_blocks<S256>(M, N, G, nprob), 256) >= f128 - 0.1 ? 3 : 1;  // (256x128 measured slower)
  }
  if (fits<S256x128>(M, N) && n_blocks<S256x128>(M, N, G, nprob) >= 256) return 2;
  return 1;
}

// layout: bit0 = A is K-major, bit1 = B is K-major.
// cfg bits 0-1: 0 = automatic shape, 1 = 128x128, 2 = 256x128, 3 = 256x256;
// bits 2-3: K pipeline (0: BK64 x 2-stage LDS ring, 1: BK32 x 4 (128x128 blocks: BK64 x 3),
// 2: BK32 x 2, 3: BK32 x 3); bit 4: 128x128 on the BK32 rings with the software-pipelined K loop.
int sc_gemm(int epi, int layout, int nprob, int M, int N, int K1, int K2, int G,
            const ScOperand* a /* [nprob][2] */, const ScOperand* b /* [nprob][2] */,
            void* const* c /* [nprob] */, const float* alpha /* [nprob] */, long ldc, long sc,
            const float* bias, long sbias, const int* nactive, const void* aux, long ldaux,
            long saux, float* part, float* colpart, const float* l1, float l1_add_scale,
            float* dotpart, int dc_tied, int cfg, int ksplit, long split_stride, void* cmask, int act, const float* ascale,
            void* cmask2, float* rcol, const int* nact_m, const int* nact_k, const int* nact_host,
            hipStream_t stream) {
  if (M % PT || N % PT || K1 % 64 || K2 % 64 || nprob < 1 || nprob > 2 || G < 1) return 1;
  if ((epi == EPI_DC_MASK || epi == EPI_DC_ACT) && !cmask) return 4;
  if (epi == EPI_DC_ACT && (!aux || !colpart || !l1)) return 4;
  if ((epi == EPI_ENC_ACT || epi == EPI_DC_ACT) && (act < 0 || act > 2 || (act == 2 && !ascale))) return 4;
  if (ksplit < 1 || ksplit > (K1 + K2) / 64 || (ksplit > 1 && epi != EPI_F32 && epi != EPI_BF16)) return 7;
  GemmParams p;
  for (int i = 0; i < nprob; ++i) {
    for (int s = 0; s < 2; ++s) {
      p.prob[i].a[s] = {reinterpret_cast<const uint16_t*>(a[i * 2 + s].ptr), a[i * 2 + s].ld, a[i * 2 + s].sg};
      p.prob[i].b[s] = {reinterpret_cast<const uint16_t*>(b[i * 2 + s].ptr), b[i * 2 + s].ld, b[i * 2 + s].sg};
    }
    p.prob[i].c = c[i];
    p.prob[i].alpha = alpha[i];
  }
  p.nprob = nprob;
  p.M = M; p.N = N; p.K1 = K1; p.K2 = K2; p.G = G;
  p.ldc = ldc; p.sc = sc;
  p.bias = bias; p.sbias = sbias; p.nactive = nactive;
  p.aux = reinterpret_cast<const uint16_t*>(aux); p.ldaux = ldaux; p.saux = saux;
  p.part = part; p.colpart = colpart; p.l1 = l1; p.l1_add_scale = l1_add_scale;
  p.dotpart = dotpart; p.dc_tied = dc_tied;
  p.cmask = reinterpret_cast<uint64_t*>(cmask);
  p.ksplit = ksplit; p.split_stride = split_stride;
  p.act = act; p.ascale = ascale;
  p.cmask2 = reinterpret_cast<uint64_t*>(cmask2); p.rcol = rcol;
  p.nact_m = nact_m; p.nact_k = nact_k;
  // masked launches with host copies of the live sizes launch only their live tiles
  p.want_comp = nact_host != nullptr && G <= 16;
  p.ncomp = 0;
  for (int g = 0; g < 16; ++g) p.nact_h[g] = (nact_host && g < G) ? nact_host[g] : 0;
  const bool ak = layout & 1, bk = layout & 2;
  int shape = cfg & 3;
  const int pipe = (cfg >> 2) & 3;  // 0: BK64 x 2 stages, 1: BK32 x 4, 2: BK32 x 2, 3: BK32 x 3
  const bool p32 = (cfg >> 4) & 1;  // 128x128 BK32 rings: the software-pipelined K loop
  // (128x256 blocks of eight 64x64 waves on the BK32 x 3 ring measured slower for the K = 512
  // step GEMMs -- 0.2914 vs 0.2886 ms/step, profiles/r5/batch5 -- and were removed)
  if (shape == 0) shape = sc_gemm_shape(M, N, G, nprob);
  switch (shape) {
    case 3:
      if (!fits<S256>(M, N)) return 6;
      return launch_big(3, pipe, epi, ak, bk, p, nprob, stream);
    case 2:
      if (!fits<S256x128>(M, N)) return 6;
      return launch_big(2, pipe, epi, ak, bk, p, nprob, stream);
    default:
      if (pipe == 1) return launch<S128, 64, 3, false>(epi, ak, bk, p, nprob, stream);  // 96 KB: 1 block/CU
      if (pipe == 2) return p32 ? launch<S128, 32, 2, false, true>(epi, ak, bk, p, nprob, stream)
                                : launch<S128, 32, 2, false>(epi, ak, bk, p, nprob, stream);  // 32 KB: 4-5 blocks/CU
      if (pipe == 3) return p32 ? launch<S128, 32, 3, false, true>(epi, ak, bk, p, nprob, stream)
                                : launch<S128, 32, 3, false>(epi, ak, bk, p, nprob, stream);
      return launch<S128, 64, 2>(epi, ak, bk, p, nprob, stream);
  }
}

}  // extern "C"
