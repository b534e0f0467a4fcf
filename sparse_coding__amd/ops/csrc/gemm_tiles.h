// Grouped-GEMM building blocks shared by the tile kernels (sae_gemm.hip) and the
// persistent tile loop (sae_gemm_kernel.h): kernel parameters, LDS image layouts, the LDS-DMA
// staging primitives and the MFMA fragment reads.  gfx950 only.
#pragma once
#include "common.h"

namespace scamd {

template <int WGM_, int WGN_, int WI_, int WJ_>
struct Shape {
  static constexpr int WGM = WGM_, WGN = WGN_, WI = WI_, WJ = WJ_;
  static constexpr int NW = WGM * WGN, NT = NW * 64;
  static constexpr int BM = WGM * WI * 16, BN = WGN * WJ * 16;
};
using S128 = Shape<2, 2, 4, 4>;
using S256x128 = Shape<2, 2, 8, 4>;
using S256x128w8 = Shape<4, 2, 4, 4>;  // 256x128 as eight 64x64 waves (two blocks per CU on BK32 x 3)
using S256 = Shape<2, 4, 8, 4>;
// Partial-sum buffers (scalar parts, column parts, row-dot parts, squared-norm
// parts) are laid out on a 128x128 sub-tile grid whatever the block shape, so the
// consumers (loss / bias / Adam kernels) do not depend on the GEMM configuration.
constexpr int PT = 128;

// (5 was EPI_ADAM, Adam fused into the weight-gradient epilogue: measured slower than the
// separate streaming Adam kernel and removed)
enum { EPI_ENC = 0, EPI_DEC = 1, EPI_DC = 2, EPI_F32 = 3, EPI_BF16 = 4, EPI_ENC_CNT = 6,
       EPI_DC_MASK = 7, EPI_ENC_ACT = 8, EPI_DC_ACT = 9, EPI_ROWMAX = 10 };

// Activity bitmask of the codes: see mask_bit() in sae_gemm_kernel.h (one 64-bit word per lane
// per 64x64 block, written by the encoder epilogue, read by the code-gradient epilogue instead
// of the bf16 codes -- 1/16 of the bytes).

// Division by a launch-constant divisor without the ~30-instruction integer-division
// sequence: q = (umulhi(n, m) + n) >> s with m, s computed on the host (round-up method,
// exact for n < 2^31).  The tile decomposition of every block is on its critical path
// (nothing is loaded until it is done), so it must be a handful of SALU ops.
struct FDiv {
  uint32_t m, s;
};
__host__ __device__ inline FDiv make_fdiv(uint32_t d) {
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  const uint64_t m = ((((1ull << s) - d) << 32) / d) + 1;
  return FDiv{(uint32_t)m, s};
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, FDiv f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

struct Operand {
  const uint16_t* ptr;
  long ld;  // leading dimension (elements)
  long sg;  // stride between groups (elements); 0 = shared by all groups
};

struct Problem {
  Operand a[2];  // two K segments (second used when k2 > 0)
  Operand b[2];
  void* c;
  float alpha;
};

struct GemmParams {
  Problem prob[2];
  int nprob;
  int M, N, K1, K2;
  int G;
  long ldc, sc;  // output leading dim / group stride (elements)
  // --- epilogue auxiliaries -------------------------------------------------
  const float* bias;  // ENC: [G][N] fp32
  long sbias;
  const int* nactive;  // ENC: per-group number of live columns (masked SAEs), may be null
  const uint16_t* aux; // DEC: x (bf16); DC: c (bf16)
  long ldaux, saux;
  float* part;         // per-block scalar partials [G][tiles] x nstat
  float* colpart;      // per-(tile_m, column) partials [G][tiles_m][N] (DC: bias grad, ENC: counts)
  const float* l1;     // DC: l1 coefficient per group
  float l1_add_scale;  // DC: multiplies l1[g] (= d/2 so dpre is in units of R)
  float* dotpart;      // DC (optional): [G][tiles_m][N] partials of the norm-Jacobian row dots
  int dc_tied;         // DC: tied dictionary -> dot also gets dpre * (c - b) (uses bias)
  uint64_t* cmask;     // ENC: optional activity-bitmask output; DC_MASK: its input
  // --- split-K (plain F32 / BF16 epilogues only): K-tile range split over `ksplit`
  // blocks per output tile; split s writes its partial product at c + s * split_stride
  // (the consumer -- the Adam kernel for weight gradients -- sums the slabs).
  int ksplit;
  long split_stride;
  // masked ensembles: per-group live extent of the n dimension when it is M / K (may be null)
  const int* nact_m;
  const int* nact_k;
  // masked decoder (nact_k only): block pairing so the two tiles that share a CU carry models g and
  // G-1-g (set by the launcher, see sae_gemm_kernel.h pair_order)
  int pair_k;
  // host-precomputed divisors of the block -> tile decomposition (set by the launcher)
  FDiv f_prob, f_split, f_plane, f_tn, f_ksplit;
  // --- EPI_ENC_ACT / EPI_DC_ACT: activation mode and the threshold SAE's per-feature s^2
  int act;
  const float* ascale;  // [G][N] (group stride sbias)
  // threshold activation (act 2): second bitmask, 1 = the code is on the ramp (u < 1),
  // decided on the fp32 pre-activation in the encoder epilogue (same layout as cmask)
  uint64_t* cmask2;
  // DEC (optional): fp32 column sums of the residual per 128-row tile [G][tiles_m][N],
  // taken before the bf16 rounding (learned-centering gradient)
  float* rcol;
  // --- masked ensembles, compacted grid (set by the launcher from host copies of the live sizes):
  // only live tiles are launched.  cdim 0: the masked dimension is N (encoder / code gradient),
  // 1: it is M (weight-gradient rows).  Model g owns tl[g] tiles along it and logical tiles
  // [tpre[g], tpre[g+1]) of each problem; fl[g] divides by tl[g].  Dead outputs are never written
  // (the engine zero-initialises them once).
  int want_comp;      // host: nact_h holds the live sizes
  int nact_h[16];
  int ncomp, cdim, ctotal;  // ctotal: live tiles per problem
  int tpre[17];
  int tl[16];
  FDiv fl[16];
};

// LDS image of a K-major tile [128 rows][BKT k] bf16.
//  BKT=64: 128-byte rows (8 chunks of 16 B), chunk ^= (row>>1)&7
//  BKT=32:  64-byte rows (4 chunks),         chunk ^= ((row>>2)&1)<<1
// Both keep the 16-lane groups of ds_read_b128 conflict free for the MFMA
// fragment reads (lane = row, chunk = k/8).
template <int BKT>
__device__ __forceinline__ int kmaj_off(int row, int ch) {
  if constexpr (BKT == 64) return row * 128 + ((ch ^ ((row >> 1) & 7)) << 4);
  else return row * 64 + ((ch ^ (((row >> 2) & 1) << 1)) << 4);
}
// LDS image of an M/N-major tile [BKT k][128 cols] bf16: 256-byte rows, 16
// chunks, swizzle that keeps the transposed 4x16 block reads conflict free.
__device__ __forceinline__ int mmaj_off(int row, int ch) {
  return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}

// s_waitcnt vmcnt(N) only (expcnt/lgkmcnt left at their maxima).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Per-lane byte offsets (relative to the operand's group base) of the 1 KiB
// LDS-DMA pieces this wave fills for K-tile 0; later tiles add a scalar soffset.
// An M/N-major tile wider than 128 is stored as 128-column halves, each its own
// [BKT][128] swizzled image (BKT/4 pieces per half).
// The LDS destination of a piece is lane-linear, so the swizzle is applied to
// the SOURCE: lane L fills physical slot L and fetches the logical chunk the
// image places there (the XOR swizzles are involutions).
template <bool KMAJ, int BKT, int PPW>
__device__ __forceinline__ void piece_offsets(uint32_t (&voff)[PPW], long ld, int r0, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int piece = wid * PPW + i;
    if constexpr (KMAJ) {
      constexpr int LPR = BKT / 8;         // lanes (16-B chunks) per row
      constexpr int RPP = 64 / LPR;        // rows per 1 KiB piece
      const int row = piece * RPP + lane / LPR;
      const int slot = lane % LPR;
      const int ch = (BKT == 64) ? (slot ^ ((row >> 1) & 7)) : (slot ^ (((row >> 2) & 1) << 1));
      // 32-bit: the buffer offset is 32-bit anyway (one group operand < 4 GiB)
      voff[i] = ((uint32_t)(r0 + row) * (uint32_t)ld + (uint32_t)(ch * 8)) * 2u;
    } else {
      constexpr int PPH = BKT / 4;  // pieces per 128-column half
      const int half = piece / PPH;
      const int row = (piece % PPH) * 4 + (lane >> 4);
      const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
      voff[i] = ((uint32_t)row * (uint32_t)ld + (uint32_t)(r0 + half * 128 + ch * 8)) * 2u;
    }
  }
}

// Buffer resource (V#) as four SGPR words for inline asm: base, stride 0,
// num_records, gfx950 raw-buffer flags.
typedef int i32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4_t make_rsrc(const uint16_t* base) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32) & 0xFFFF);
  r[2] = 0x7FFFFFFF;
  r[3] = 0x00020000;
  return r;
}

// The LDS-DMA is issued from inline asm on purpose: when hipcc sees a
// buffer_load...lds it conservatively waits vmcnt(0) before the next ds_read of
// the same LDS array, which would drain the prefetch of tile kt+1 before tile
// kt's MFMAs and serialise the pipeline.  Hidden in asm, the DMAs are waited for
// only by the explicit counted vmcnt before each barrier.
template <int PPW>
__device__ __forceinline__ void issue_pieces(const i32x4_t& rs, const uint32_t* voff, uint32_t soff, char* lds_tile,
                                             int wid) {
  const uint32_t base = (uint32_t)reinterpret_cast<uintptr_t>(lds_tile) + (uint32_t)(wid * PPW * 1024);
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    asm volatile(
        "s_mov_b32 m0, %0\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, %3 offen lds"
        :
        : "s"(base + i * 1024), "v"(voff[i]), "s"(rs), "s"(soff)
        : "memory", "m0");
  }
}

// Fragment for v_mfma_f32_16x16x32_bf16: lane l holds X[r = rbase + (l&15)][k = 32 ks + 8(l>>4) + j].
template <bool KMAJ, int BKT>
__device__ __forceinline__ bf16x8_t load_frag(const char* lds, int rbase, int ks, int lane) {
  if constexpr (KMAJ) {
    const int row = rbase + (lane & 15);
    const int ch = ks * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8_t*>(lds + kmaj_off<BKT>(row, ch));
  } else {
    // ds_read_b64_tr_b16: lane 4q+p of each 16-lane group addresses row q,
    // columns 4p..4p+3 of a 4x16 block; lane i receives column i.
    lds += (rbase >> 7) * (BKT * 256);  // 128-column half image
    rbase &= 127;
    const int li = lane & 15, q = li >> 2, p = li & 3, g = lane >> 4;
    const int ch = (rbase >> 3) + (p >> 1);
    const int within = (p & 1) * 8;
    const int row0 = ks * 32 + 8 * g + q;
    i16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(SC_LDS(i16x4_t, lds + mmaj_off(row0, ch) + within));
    i16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(SC_LDS(i16x4_t, lds + mmaj_off(row0 + 4, ch) + within));
    typedef short i16x8_t __attribute__((ext_vector_type(8)));
    i16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
}


}  // namespace scamd
