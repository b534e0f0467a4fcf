// Grouped bf16 MFMA GEMM with fused sparse-autoencoder epilogues (gfx950).
//
// One launch covers every model of an ensemble (the "group" axis G) and, for
// the weight-gradient pass, two independent problems at once.  This replaces
// the reference's torch.vmap(torch.func.grad(loss)) over stacked parameters
// (reference autoencoders/ensemble.py:119-123) with explicit kernels:
//
//   EPI_ENC : c = relu(x W_e^T + b)  (+ masked tail), bf16 store, L1/L0 partials
//   EPI_ENC_CNT: EPI_ENC + per-feature fire counts (a separate instantiation: the
//             count reduction costs ~10% of the kernel and runs only on sampled steps)
//             (autoencoders/sae_ensemble.py:54-56, :354 masked_fill_)
//   EPI_DEC : R = c W_hat - x, bf16 store, sum(R^2) partials
//             (autoencoders/sae_ensemble.py:58-62)
//   EPI_DC  : dpre_s = 1[c>0] * (R W_hat^T + lambda*d/2), bf16 store, column-sum
//             partials for the bias gradient (autograd of :54-64, Appendix A of SURVEY)
//   EPI_F32 : C = alpha * acc (fp32), used for dW = c^T R and dW_e = dpre^T x
//   EPI_BF16: C = alpha * acc (bf16), generic inference GEMM
//   EPI_ENC_ACT / EPI_DC_ACT: EPI_ENC / EPI_DC_MASK for the other code activations
//             (GemmParams::act): 1 = reverse SAE, codes 1[pre > 0] (pre - b)
//             (sae_ensemble.py:481-482); 2 = smooth threshold
//             s^2 thr((pre)/s^2), thr(u) = relu6(60(u - 0.9))/6 + relu(u - 1) (:254-257)
//   EPI_ROWMAX: per-row max of alpha * A B^T over column tiles (max cosine similarity /
//             MMCS, standard_metrics.py:268-301) -- the [M, N] product never reaches HBM
//
// Tiling (template "shape"): a WGM x WGN grid of waves, each owning a
// (16 WI) x (16 WJ) sub-tile = WI x WJ v_mfma_f32_16x16x32_bf16 accumulators:
//   S128   : 2x2 waves of 64x64   -> 128x128 block, 256 threads
//   S256x128: 2x2 waves of 128x64 -> 256x128 block, 256 threads
//   S256   : 2x4 waves of 128x64  -> 256x256 block, 512 threads, 1 block/CU
// Bigger tiles raise FLOPs per staged byte (64 -> 85 -> 128 FLOP/B) and per LDS
// fragment read (per-wave 128x64 reads 12 fragments per 32 MFMAs instead of 8 per
// 16), which is what limits the short-K (K = d = 512) step GEMMs.  Operands
// are staged global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds) into an
// NST-deep ring of BKT-deep K-tiles (configurations: BK64 x 2 stages, BK32 x 3
// or 4 stages).  Per-lane source offsets are computed once; the K loop only
// advances a scalar soffset, so the main loop is MFMA + ds_read + a handful of
// SALU.  One raw s_barrier per K-tile with a counted vmcnt keeps NST-2 tiles in
// flight across it.
// K-major operands are read with ds_read_b128, M/N-major operands with the
// gfx950 transposing read ds_read_b64_tr_b16, so c^T R style products need no
// transposed copies in HBM.  Both LDS images are XOR-swizzled to avoid bank
// conflicts.
//
// This header holds the kernel template and its launcher; two translation units
// instantiate it: sae_gemm.hip (128x128 blocks, built with the VGPR form of the MFMA
// for the software-pipelined K loop) and sae_gemm_big.hip (256x128 / 256x256 blocks,
// AGPR accumulators: at 128 accumulator registers per wave the VGPR form spills).
#pragma once
#include "gemm_tiles.h"

#include <algorithm>
#include <stdlib.h>

namespace scamd {

// Scheduling-group pattern for one pipelined K-step: N x (MPR MFMAs, then one DS read), the
// last group taking LASTM MFMAs.  An MFMA leads so the step's first MFMA never sits behind a
// read just issued (at the loop header the waitcnt pass falls back to lgkmcnt(0)).
// (sched_group_barrier needs literal arguments, hence the recursion.)
template <int N, int MPR, int LASTM>
__device__ __forceinline__ void sched_interleave() {
  if constexpr (N > 0) {
    __builtin_amdgcn_sched_group_barrier(0x008, N == 1 ? LASTM : MPR, 0);  // MFMAs
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                    // one DS read
    sched_interleave<N - 1, MPR, LASTM>();
  }
}

// ------------------------------------------------------------------ code activity bitmask
// Layout [G][B/64][n/64][64 lanes] uint64: within each 64x64 block of the codes, lane l owns
// the 64 elements it holds in the MFMA output layout -- rows 16 ii + (l & 15), columns
// 16 jj + 4 (l >> 4) + r for ii, jj, r in 0..3 -- as bit (4 ii + jj) * 4 + r.  Any wave
// sub-tile made of 64x64 blocks (64x64 at 128x128 blocks, 128x64 at 256-row blocks) writes
// and reads it with one 8-byte access per lane per block: no ballots, no lane-0 scatter.
__device__ __forceinline__ constexpr int mask_bit(int i, int j, int r) { return (((i & 3) * 4 + j) * 4 + r); }
__device__ __forceinline__ bool mask_get(uint64_t w, int i, int j, int r) { return (w >> mask_bit(i, j, r)) & 1ull; }
// word index of the 64x64 block at (row0, col0) (multiples of 64) for this lane
__device__ __forceinline__ long mask_word(const GemmParams& p, int g, int row0, int col0, int lane) {
  return (((long)g * (p.M >> 6) + (row0 >> 6)) * (p.N >> 6) + (col0 >> 6)) * 64 + lane;
}

// ------------------------------------------------------------------ phase stamps (lab builds only)
// scripts/lab/gemm_phases.hip defines SC_PHASE_STAMPS to time the phases of every workgroup
// (start, first K-tile landed, K loop done, epilogue done) into a buffer of its own; product
// builds compile these to nothing.
#ifdef SC_PHASE_STAMPS
__device__ long long* sc_stamp_buf;
// volatile asm: the builtins are free to be scheduled (and merged) anywhere in the kernel
__device__ __forceinline__ long long sc_memtime() {
  long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  return t;
}
__device__ __forceinline__ long long sc_memrealtime() {
  long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  return t;
}
#define SC_STAMP(k)                                                                      \
  do {                                                                                   \
    if (threadIdx.x == 0 && sc_stamp_buf) {                                              \
      long long* st_ = sc_stamp_buf + (long)blockIdx.x * 8;                              \
      st_[k] = sc_memtime();                                                             \
      if ((k) == 0) {                                                                    \
        st_[4] = sc_memrealtime();                                                       \
        st_[6] = (long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);                   \
        st_[7] = (long long)__builtin_amdgcn_s_getreg((15 << 11) | 20);                  \
      }                                                                                  \
      if ((k) == 3) st_[5] = sc_memrealtime();                                           \
    }                                                                                    \
  } while (0)
// sub-phases of the epilogue (wave 0's view), same lab builds: slots [block][8] of sc_sub_buf
__device__ long long* sc_sub_buf;
#define SC_SUB(k)                                                                          \
  do {                                                                                     \
    if (threadIdx.x == 0 && sc_sub_buf) sc_sub_buf[(long)blockIdx.x * 8 + (k)] = sc_memtime(); \
  } while (0)
#else
#define SC_STAMP(k) do {} while (0)
#define SC_SUB(k) do {} while (0)
#endif

// ------------------------------------------------------------------ epilogues
// The fused epilogue of one output tile (shared by the tile kernel and the persistent
// kernel).  `red` is LDS scratch of at least epi_scratch_floats<S>() floats; every
// barrier in here is LDS-only (lgkmcnt(0) + s_barrier), so in-flight global stores and
// LDS-DMA prefetches of a persistent block are not drained.
template <class S>
constexpr int epi_scratch_floats() { return 2 * S::WGM * S::BN + 2 * S::NW; }

// LDS-staged bf16 output stores (STAGE, 128x128 tile kernel: the ring is free after the K
// loop): each wave parks its 64x64 bf16 sub-tile in LDS in the MFMA layout, then streams it
// out row-contiguous -- 8 global_store_dwordx4 per wave, each covering 8 whole 128-byte row
// segments, instead of 16 dwordx2 stores that each touch 16 half-filled 32-byte segments (the
// store tail is issue-bound otherwise).  Rows are 128 bytes; the 16-byte chunk index is XORed
// with (row >> 1) & 7 and the two 8-byte halves of a chunk swap on odd rows.  Banking per
// instruction (MI355X_MICROARCH.md, LDS): ds_write_b64 serves 16 contiguous lanes at a time on
// 32 banks -- a group is 16 rows at one column, and the chunk XOR alone gives only 8 distinct
// bank pairs (2-way, measured: 64 extra cycles per wave); the half swap makes them 16.
// ds_read_b128 serves 16-lane groups on 64 banks: 2 rows x 8 chunks, distinct with the XOR.
constexpr int STAGE_OFF = 4096, STAGE_ROW = 128;
template <class S>
constexpr int stage_wave() { return S::WI * 16 * STAGE_ROW; }  // a wave's (16 WI) x 64 bf16 sub-tile
__device__ __forceinline__ int stage_at(int row, int byte) {  // 8-byte granule of (row, byte)
  return row * STAGE_ROW + ((((byte >> 4) ^ (row >> 1)) & 7) << 4) + ((((byte >> 3) ^ row) & 1) << 3);
}
template <class S>
constexpr int stage_off() { return ((2 * S::WGM * S::BN + 2 * S::NW) * 4 + STAGE_OFF - 1) / STAGE_OFF * STAGE_OFF; }
template <class S>
constexpr int stage_bytes() { return stage_off<S>() + S::NW * stage_wave<S>(); }

template <class S, int EPI, bool AUX_EARLY, bool STAGE = false, bool FSTAGE = false>
__device__ __forceinline__ void sae_epilogue(const GemmParams& p, f32x4_t (&acc)[S::WI][S::WJ],
                                             const uint2 (&auxv)[S::WI][S::WJ], const f32x4_t (&biasv)[S::WJ],
                                             const uint64_t (&mkv)[S::WI / 4],
                                             float* red, int pi, int g, int m0, int n0, int tn, int tiles_n,
                                             void* cptr, float alpha, bool dead = false) {
  constexpr int BM = S::BM, BN = S::BN, NT = S::NT, NW = S::NW, WI = S::WI, WJ = S::WJ, WGN = S::WGN;
  constexpr bool ENC = (EPI == EPI_ENC || EPI == EPI_ENC_CNT || EPI == EPI_ENC_ACT);
  constexpr int RED_SUM = 2 * S::WGM * BN;  // block_sum scratch after the two column-sum regions
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WGN, wc = wid % WGN;
  const int ptm = p.M / PT, ptn = p.N / PT;
  const bool p1 = pi != 0;
  const int rowb = m0 + wr * (WI * 16) + (lane & 15);
  const int colb = n0 + wc * (WJ * 16) + 4 * (lane >> 4);
  static_assert(!STAGE || ((WI == 4 || WI == 8) && WJ == 4 && 2 * S::WGM * BN + 2 * NW <= stage_off<S>() / 4),
                "stage layout");
  char* stage = reinterpret_cast<char*>(red) + stage_off<S>() + wid * stage_wave<S>();
  // one 4-wide bf16 output fragment (rows rowb + 16 i, columns colb + 16 j .. +3)
  auto put = [&](uint16_t* C, int i, int j, ushort4 h) {
    if constexpr (STAGE) {
      *reinterpret_cast<ushort4*>(stage + stage_at(i * 16 + (lane & 15), (j * 16 + 4 * (lane >> 4)) * 2)) = h;
    } else {
      *reinterpret_cast<ushort4*>(C + (long)(rowb + i * 16) * p.ldc + colb + j * 16) = h;
    }
  };
  auto flush = [&](uint16_t* C) {
    if constexpr (STAGE) {  // (one wave's LDS ops complete in order: no barrier needed)
      uint16_t* Cw = C + (long)(m0 + wr * (WI * 16)) * p.ldc + n0 + wc * (WJ * 16);
      const int ch = lane & 7;
#pragma unroll
      for (int k = 0; k < 2 * WI; ++k) {
        const int row = 8 * k + (lane >> 3);
        uint4 v = *reinterpret_cast<const uint4*>(stage + row * STAGE_ROW + (((ch ^ (row >> 1)) & 7) << 4));
        if (row & 1) v = make_uint4(v.z, v.w, v.x, v.y);  // halves stored swapped on odd rows
        *reinterpret_cast<uint4*>(Cw + (long)row * p.ldc + ch * 8) = v;
      }
    }
  };

  constexpr bool CAN_DIE = ENC || EPI == EPI_DC || EPI == EPI_DC_MASK || EPI == EPI_DC_ACT || EPI == EPI_F32;
  if (CAN_DIE && dead) {
    // A tile wholly past a model's live dictionary (masked ensembles): no MFMA work ran.  The
    // encoder still writes its zero codes and activity words and the weight gradient its
    // zero rows (API outputs); the code gradient's dead columns are left unwritten (only the
    // engine passes nactive there, and nothing downstream reads them: the weight gradient
    // skips those rows); the partial sums consumers add over every tile are zeroed.
    if constexpr (ENC) {
      uint16_t* C = reinterpret_cast<uint16_t*>(cptr) + (long)g * p.sc;
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int j = 0; j < WJ; ++j)
          *reinterpret_cast<ushort4*>(C + (long)(rowb + i * 16) * p.ldc + colb + j * 16) = make_ushort4(0, 0, 0, 0);
      if (p.cmask) {
#pragma unroll
        for (int k = 0; k < WI / 4; ++k) {
          const long w = mask_word(p, g, rowb - (lane & 15) + 64 * k, colb - 4 * (lane >> 4), lane);
          p.cmask[w] = 0ull;
          if (p.cmask2) p.cmask2[w] = 0ull;
        }
      }
    }
    if constexpr (EPI == EPI_F32) {
      float* C = reinterpret_cast<float*>(cptr) + (long)g * p.sc;
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int j = 0; j < WJ; ++j)
          *reinterpret_cast<f32x4_t*>(C + (long)(rowb + i * 16) * p.ldc + colb + j * 16) = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (ENC) {
      for (int idx = tid; idx < (BM / PT) * (BN / PT); idx += NT) {
        const int sm = idx / (BN / PT), sn = idx - sm * (BN / PT);
        float* dst = p.part + ((long)g * ptm * ptn + (m0 / PT + sm) * ptn + n0 / PT + sn) * 2;
        dst[0] = 0.f;
        dst[1] = 0.f;
      }
    }
    if constexpr (ENC || EPI == EPI_DC || EPI == EPI_DC_MASK || EPI == EPI_DC_ACT) {
      float* outs[2] = {p.colpart, (EPI == EPI_DC || EPI == EPI_DC_ACT) ? p.dotpart : nullptr};
#pragma unroll
      for (int o = 0; o < 2; ++o) {
        if (!outs[o]) continue;
        for (int idx = tid; idx < (BM / PT) * BN; idx += NT) {
          const int sl = idx / BN, col = idx - sl * BN;
          outs[o][((long)g * ptm + m0 / PT + sl) * p.N + n0 + col] = 0.f;
        }
      }
    }
    return;
  }

  if constexpr (EPI == EPI_F32) {
    float* C = reinterpret_cast<float*>(cptr) + (long)g * p.sc;
    if constexpr (FSTAGE) {
      // LDS-staged row-contiguous fp32 stores (tile kernel, ring free after the K loop): the
      // MFMA layout puts 16 rows x 64 B in one store; instead each wave parks 32 columns of
      // its sub-tile (128-byte rows, the bf16 staging's swizzle) and streams whole 128-byte
      // row segments, 8 rows per dwordx4 store; two passes cover the 64 columns.
      char* st = reinterpret_cast<char*>(red) + wid * (WI * 16 * STAGE_ROW);
      float* Cw = C + (long)(m0 + wr * (WI * 16)) * p.ldc + n0 + wc * (WJ * 16);
      const int q = lane >> 4, r16 = lane & 15, ch = lane & 7;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < WI; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const f32x4_t v = acc[i][2 * h + jj] * alpha;
            const int row = i * 16 + r16, byte = (jj * 16 + 4 * q) * 4;
            *reinterpret_cast<float2*>(st + stage_at(row, byte)) = make_float2(v[0], v[1]);
            *reinterpret_cast<float2*>(st + stage_at(row, byte + 8)) = make_float2(v[2], v[3]);
          }
#pragma unroll
        for (int k = 0; k < WI * 2; ++k) {
          const int row = 8 * k + (lane >> 3);
          uint4 u = *reinterpret_cast<const uint4*>(st + row * STAGE_ROW + (((ch ^ (row >> 1)) & 7) << 4));
          if (row & 1) u = make_uint4(u.z, u.w, u.x, u.y);
          *reinterpret_cast<uint4*>(Cw + (long)row * p.ldc + h * 32 + ch * 4) = u;
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
      for (int j = 0; j < WJ; ++j) {
        const f32x4_t v = acc[i][j] * alpha;
        *reinterpret_cast<f32x4_t*>(C + (long)(rowb + i * 16) * p.ldc + colb + j * 16) = v;
      }
    return;
  }
  if constexpr (EPI == EPI_BF16) {
    uint16_t* C = reinterpret_cast<uint16_t*>(cptr) + (long)g * p.sc;
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
      for (int j = 0; j < WJ; ++j) {
        ushort4 h;
        h.x = f2bf(alpha * acc[i][j][0]); h.y = f2bf(alpha * acc[i][j][1]);
        h.z = f2bf(alpha * acc[i][j][2]); h.w = f2bf(alpha * acc[i][j][3]);
        put(C, i, j, h);
      }
    flush(C);
    return;
  }
  // Column partial sums (ENC: on-counts, DC: bias gradient) per 128-row slot, in
  // two steps so no per-column array stays live across the epilogue: (1) right
  // after fragment column j is produced, reduce its 4 columns over the lane's
  // rows and the 16 lanes sharing them (xor shuffles) and park the result in LDS
  // (region `slot` of `red`); (2) after a barrier, sum the wave rows of each
  // 128-row slot and store one value per (slot, column).  Deterministic.
  constexpr int WPS = PT / (WI * 16);  // wave rows per 128-row slot
  auto colred_lane = [&](f32x4_t v, int j, int region) {
    // sum over the 16 lanes of a DPP row (the fragment's 16 output rows): lane 15 ends
    // with the total -- four DPP adds per value instead of four ds_bpermute shuffles
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = row16_scan(v[r]);
    if ((lane & 15) == 15)
      *reinterpret_cast<f32x4_t*>(red + region * (S::WGM * BN) + wr * BN + wc * (WJ * 16) + j * 16 +
                                  4 * (lane >> 4)) = v;
  };
  auto colred_store = [&](float* dst, int region) {
    const float* rr = red + region * (S::WGM * BN);
    for (int idx = tid; idx < (BM / PT) * BN; idx += NT) {
      const int s = idx / BN, col = idx - s * BN;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < WPS; ++w) v += rr[(s * WPS + w) * BN + col];
      dst[((long)g * ptm + m0 / PT + s) * p.N + n0 + col] = v;
    }
  };
  // Scalar partials live on the 128x128 grid: the block total goes to its first
  // sub-tile, the block's other sub-tiles get zero (consumers sum them all).
  auto scalar_partial = [&](float* base, int nstat, int stat, float v) {
    if (tid < (BM / PT) * (BN / PT)) {
      const int sm = tid / (BN / PT), sn = tid - sm * (BN / PT);
      base[((long)g * ptm * ptn + (m0 / PT + sm) * ptn + n0 / PT + sn) * nstat + stat] = tid == 0 ? v : 0.f;
    }
  };

  if constexpr (ENC) {
    SC_SUB(0);
    uint16_t* C = reinterpret_cast<uint16_t*>(cptr) + (long)g * p.sc;
    const float* bias = p.bias + (long)g * p.sbias;
    const int nact = p.nactive ? p.nactive[g] : p.N;  // masked SAEs: live columns [0, nact)
    constexpr bool ACTV = EPI == EPI_ENC_ACT;
    const int act = ACTV ? p.act : 0;  // compile-time 0 for the plain ReLU instantiations
    const bool counting = EPI == EPI_ENC_CNT || (ACTV && p.colpart != nullptr);
    // 128x128 blocks: column masking only where the block reaches past nactive (uniform
    // branch); L0 from the activity ballots' popcounts (scalar) whenever they are taken
    const bool full = WI * WJ <= 16 && nact >= n0 + BN;
    const bool l0_from_mask = !ACTV && EPI != EPI_ENC_CNT && p.cmask != nullptr;
    float l1 = 0.f, l0 = 0.f;
    // activity / ramp bitmask words of this lane, one 64-bit word per 64x64 block (mask_bit)
    uint32_t mw[WI / 4][2], qw[WI / 4][2];
#pragma unroll
    for (int k = 0; k < WI / 4; ++k) mw[k][0] = mw[k][1] = qw[k][0] = qw[k][1] = 0u;
#pragma unroll
    for (int j = 0; j < WJ; ++j) {
      const int col = colb + j * 16;
      const f32x4_t bj = ACTV ? *reinterpret_cast<const f32x4_t*>(bias + col) : biasv[j];  // (ReLU: loaded before the K loop)
      f32x4_t s2 = f32x4_t{1.f, 1.f, 1.f, 1.f}, is2 = s2;
      if (ACTV && act == 2) {
        s2 = *reinterpret_cast<const f32x4_t*>(p.ascale + (long)g * p.sbias + col);
#pragma unroll
        for (int r = 0; r < 4; ++r) is2[r] = 1.f / fmaxf(s2[r], 1e-8f);
      }
      f32x4_t cnt = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < WI; ++i) {
        f32x4_t v;
        bool on[4], rampv[4] = {false, false, false, false};
        if constexpr (ACTV) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float pre = acc[i][j][r] + bj[r];
            if (act == 1) {
              v[r] = pre > 0.f ? acc[i][j][r] : 0.f;  // relu(pre) - b on the active codes
            } else if (act == 2) {
              const float u = pre * is2[r];
              v[r] = (fminf(fmaxf(10.f * (u - 0.9f), 0.f), 1.f) + fmaxf(u - 1.f, 0.f)) * s2[r];
              rampv[r] = u < 1.f;
            } else {
              v[r] = fmaxf(pre, 0.f);
            }
            const bool live = col + r < nact;
            on[r] = live && (act == 1 ? pre > 0.f : v[r] > 0.f);
            rampv[r] = rampv[r] && on[r];
            v[r] = live ? v[r] : 0.f;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            l1 += fabsf(v[r]);
            const float onf = on[r] ? 1.f : 0.f;
            l0 += onf;
            cnt[r] += onf;
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(acc[i][j][r] + bj[r], 0.f);
          // (128x64-per-wave blocks stay branch-free: a block-uniform `if (masked)` made hipcc
          // version the whole epilogue and spill there)
          if (!full) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (col + r < nact) ? v[r] : 0.f;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            l1 += v[r];
            on[r] = v[r] > 0.f;
          }
          if (!l0_from_mask) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float onf = on[r] ? 1.f : 0.f;
              l0 += onf;
              cnt[r] += onf;
            }
          }
        }
        put(C, i, j, make_ushort4(f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])));
        if (p.cmask) {  // block-uniform: set this lane's bits (compile-time positions)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int bit = mask_bit(i, j, r);
            mw[i / 4][bit >> 5] |= on[r] ? (1u << (bit & 31)) : 0u;
            if (ACTV) qw[i / 4][bit >> 5] |= rampv[r] ? (1u << (bit & 31)) : 0u;
          }
        }
      }
      if (counting) colred_lane(cnt, j, 0);
    }
    SC_SUB(1);
    flush(C);
    SC_SUB(2);
    if (p.cmask) {
#pragma unroll
      for (int k = 0; k < WI / 4; ++k) {
        const long w = mask_word(p, g, rowb - (lane & 15) + 64 * k, colb - 4 * (lane >> 4), lane);
        p.cmask[w] = ((uint64_t)mw[k][1] << 32) | mw[k][0];
        if (ACTV && act == 2 && p.cmask2) p.cmask2[w] = ((uint64_t)qw[k][1] << 32) | qw[k][0];
        if (l0_from_mask) l0 += (float)(__popc(mw[k][0]) + __popc(mw[k][1]));
      }
    }
    SC_SUB(3);
    // one barrier: publishes the colred_lane writes too; `red` is not written after it
    const float2 sums = block_sum2_final<NW>(l1, l0, red + RED_SUM);
    l1 = sums.x;
    l0 = sums.y;
    SC_SUB(4);
    if (counting) colred_store(p.colpart, 0);
    scalar_partial(p.part, 2, 0, l1);
    scalar_partial(p.part, 2, 1, l0);
    SC_SUB(5);
    return;
  }
  if constexpr (EPI == EPI_DEC) {
    uint16_t* C = reinterpret_cast<uint16_t*>(cptr) + (long)g * p.sc;
    float se = 0.f;
    const bool rcol = p.rcol != nullptr;  // fp32 column sums of R (learned-centering gradient)
#pragma unroll
    for (int j = 0; j < WJ; ++j) {
      f32x4_t cs = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < WI; ++i) {
        const long row = rowb + i * 16;
        const int col = colb + j * 16;
        const uint2 xv = AUX_EARLY ? auxv[i][j]
                                   : *reinterpret_cast<const uint2*>(p.aux + (long)g * p.saux + row * p.ldaux + col);
        const float r0 = acc[i][j][0] - bf2f(xv.x & 0xFFFF), r1 = acc[i][j][1] - bf2f(xv.x >> 16);
        const float r2 = acc[i][j][2] - bf2f(xv.y & 0xFFFF), r3 = acc[i][j][3] - bf2f(xv.y >> 16);
        put(C, i, j, make_ushort4(f2bf(r0), f2bf(r1), f2bf(r2), f2bf(r3)));
        se += r0 * r0 + r1 * r1 + r2 * r2 + r3 * r3;
        cs[0] += r0; cs[1] += r1; cs[2] += r2; cs[3] += r3;
      }
      if (rcol) colred_lane(cs, j, 0);
    }
    flush(C);
    se = block_sum2_final<NW>(se, 0.f, red + RED_SUM).x;  // its barrier also publishes colred_lane's writes
    if (rcol) colred_store(p.rcol, 0);
    scalar_partial(p.part, 1, 0, se);
    return;
  }
  if constexpr (EPI == EPI_DC) {
    uint16_t* C = reinterpret_cast<uint16_t*>(cptr) + (long)g * p.sc;
    const float add = p.l1[g] * p.l1_add_scale;
    const bool want_dot = p.dotpart != nullptr;
#pragma unroll
    for (int j = 0; j < WJ; ++j) {
      f32x4_t cs = f32x4_t{0.f, 0.f, 0.f, 0.f}, ds = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int col = colb + j * 16;
      f32x4_t bj = f32x4_t{0.f, 0.f, 0.f, 0.f};
      if (p.dc_tied) bj = *reinterpret_cast<const f32x4_t*>(p.bias + (long)g * p.sbias + col);
#pragma unroll
      for (int i = 0; i < WI; ++i) {
        const long row = rowb + i * 16;
        const uint2 cv = AUX_EARLY ? auxv[i][j]
                                   : *reinterpret_cast<const uint2*>(p.aux + (long)g * p.saux + row * p.ldaux + col);
        const uint16_t cvs[4] = {(uint16_t)(cv.x & 0xFFFF), (uint16_t)(cv.x >> 16), (uint16_t)(cv.y & 0xFFFF),
                                 (uint16_t)(cv.y >> 16)};
        f32x4_t dv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float c = bf2f(cvs[r]);
          dv[r] = c > 0.f ? acc[i][j][r] + add : 0.f;  // c is a ReLU output
          cs[r] += dv[r];
          if (want_dot) {
            // <w_hat_j, dL/dw_hat_j> (in units of 2/(B d)): decoder path c * (R w_hat^T),
            // tied encoder path dpre * (x w_hat^T) = dpre * (pre - b) = dpre * (c - b)
            ds[r] += c * acc[i][j][r] + (p.dc_tied ? dv[r] * (c - bj[r]) : 0.f);
          }
        }
        put(C, i, j, make_ushort4(f2bf(dv[0]), f2bf(dv[1]), f2bf(dv[2]), f2bf(dv[3])));
      }
      colred_lane(cs, j, 0);
      if (want_dot) colred_lane(ds, j, 1);
    }
    flush(C);
    lds_barrier();
    colred_store(p.colpart, 0);
    if (want_dot) colred_store(p.dotpart, 1);
    return;
  }
  if constexpr (EPI == EPI_DC_MASK) {
    // EPI_DC with the code activity read from the encoder's bitmask (no norm-Jacobian dots)
    uint16_t* C = reinterpret_cast<uint16_t*>(cptr) + (long)g * p.sc;
    const float add = p.l1[g] * p.l1_add_scale;
    const uint64_t (&mk)[WI / 4] = mkv;  // this lane's activity words, fetched before the K loop
#pragma unroll
    for (int j = 0; j < WJ; ++j) {
      f32x4_t cs = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int col = colb + j * 16;
#pragma unroll
      for (int i = 0; i < WI; ++i) {
        const long row = rowb + i * 16;
        f32x4_t dv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool on = mask_get(mk[i / 4], i, j, r);
          dv[r] = on ? acc[i][j][r] + add : 0.f;
          cs[r] += dv[r];
        }
        put(C, i, j, make_ushort4(f2bf(dv[0]), f2bf(dv[1]), f2bf(dv[2]), f2bf(dv[3])));
      }
      colred_lane(cs, j, 0);
    }
    flush(C);
    lds_barrier();
    colred_store(p.colpart, 0);
    return;
  }
  if constexpr (EPI == EPI_DC_ACT) {
    // Code gradient of the reverse / threshold activations: activity from the encoder's
    // bitmask, the codes themselves (aux) for the L1 sign (reverse codes can be negative)
    // and the threshold's slope.  Threshold: thr' = 10 on the ramp (c / s^2 < 1), 1 above;
    // region 1 collects sum_b dL/dc * (thr - u thr') = -9 dL/dc on the ramp (the s^2
    // gradient: dL/ds = 2 s * that); reverse SAEs get no bias gradient (column sums 0).
    uint16_t* C = reinterpret_cast<uint16_t*>(cptr) + (long)g * p.sc;
    const float add = p.l1[g] * p.l1_add_scale;
    const int act = p.act;
    uint64_t mk[WI / 4], rk[WI / 4];  // activity / ramp words of this lane
#pragma unroll
    for (int k = 0; k < WI / 4; ++k) {
      const long w = mask_word(p, g, rowb - (lane & 15) + 64 * k, colb - 4 * (lane >> 4), lane);
      mk[k] = p.cmask[w];
      rk[k] = p.cmask2 ? p.cmask2[w] : 0ull;
    }
#pragma unroll
    for (int j = 0; j < WJ; ++j) {
      f32x4_t cs = f32x4_t{0.f, 0.f, 0.f, 0.f}, ds = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int col = colb + j * 16;
      f32x4_t is2 = f32x4_t{1.f, 1.f, 1.f, 1.f};
      if (act == 2) {
        const f32x4_t s2 = *reinterpret_cast<const f32x4_t*>(p.ascale + (long)g * p.sbias + col);
#pragma unroll
        for (int r = 0; r < 4; ++r) is2[r] = 1.f / fmaxf(s2[r], 1e-8f);
      }
#pragma unroll
      for (int i = 0; i < WI; ++i) {
        const long row = rowb + i * 16;

        const uint2 cv = AUX_EARLY ? auxv[i][j]
                                   : *reinterpret_cast<const uint2*>(p.aux + (long)g * p.saux + row * p.ldaux + col);
        const uint16_t cvs[4] = {(uint16_t)(cv.x & 0xFFFF), (uint16_t)(cv.x >> 16), (uint16_t)(cv.y & 0xFFFF),
                                 (uint16_t)(cv.y >> 16)};
        f32x4_t dv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool on = mask_get(mk[i / 4], i, j, r);
          const float c = bf2f(cvs[r]);
          if (act == 1) {
            const float sgn = c > 0.f ? 1.f : (c < 0.f ? -1.f : 0.f);
            dv[r] = on ? acc[i][j][r] + add * sgn : 0.f;
          } else if (act == 2) {
            const float dc = acc[i][j][r] + add;
            // ramp bit from the encoder's fp32 decision; without it, from the bf16 code
            const bool ramp = p.cmask2 ? mask_get(rk[i / 4], i, j, r) : c * is2[r] < 1.f;
            dv[r] = on ? dc * (ramp ? 10.f : 1.f) : 0.f;
            cs[r] += dv[r];
            ds[r] += (on && ramp) ? -9.f * dc : 0.f;
          } else {
            dv[r] = on ? acc[i][j][r] + add : 0.f;
            cs[r] += dv[r];
          }
        }
        put(C, i, j, make_ushort4(f2bf(dv[0]), f2bf(dv[1]), f2bf(dv[2]), f2bf(dv[3])));
      }
      colred_lane(cs, j, 0);
      colred_lane(ds, j, 1);
    }
    flush(C);
    lds_barrier();
    colred_store(p.colpart, 0);
    if (p.dotpart) colred_store(p.dotpart, 1);
    return;
  }
  if constexpr (EPI == EPI_ROWMAX) {
    // max over this wave's columns of each output row, then over the four 16-lane groups
    // holding the same row; one partial per (row, wave column) -> C[g][row][tn * WGN + wc]
    float* C = reinterpret_cast<float*>(cptr) + (long)g * p.sc;
    const long ldp = (long)tiles_n * WGN;
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      float mx = -3.0e38f;
#pragma unroll
      for (int j = 0; j < WJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, alpha * acc[i][j][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 16));
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      if (lane < 16) C[(long)(rowb + i * 16) * ldp + tn * WGN + wc] = mx;
    }
    return;
  }
}

// One output tile (logical block `bid`) of a grouped GEMM launch, with its LDS ring at `smem`.
template <class S, bool AK, bool BKM, int EPI, int BKT, int NST, bool P32 = false>
__device__ __forceinline__ void gemm_block(const GemmParams& p, const int bid, char* smem) {
  constexpr int BM = S::BM, BN = S::BN, NT = S::NT, NW = S::NW, WI = S::WI, WJ = S::WJ, WGN = S::WGN;
  constexpr int TA = BM * BKT * 2, TBB = BN * BKT * 2;  // bytes per operand tile
  constexpr int PPWA = TA / 1024 / NW, PPWB = TBB / 1024 / NW;  // LDS-DMA pieces per wave
  constexpr int LPT = PPWA + PPWB;                       // DMA instructions per wave per K-tile
  constexpr int STG = TA + TBB;
  static_assert(PPWA * NW * 1024 == TA && PPWB * NW * 1024 == TBB, "tile must split into whole pieces");
  SC_STAMP(0);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WGN, wc = wid % WGN;
  const int tiles_m = p.M / BM, tiles_n = p.N / BN;
  const int ptm = p.M / PT, ptn = p.N / PT;  // partial-buffer grid (128 x 128 sub-tiles)
  const int per_split = p.ncomp ? p.ctotal : tiles_m * tiles_n * p.G;
  const int per_prob = per_split * p.ksplit;
  const int pi = (int)fdiv(bid, p.f_prob);
  int rem = bid - pi * per_prob;
  const int ksi = (int)fdiv(rem, p.f_split);
  rem -= ksi * per_split;
  int g, tm, tn;
  if (p.ncomp) {
    // compacted masked grid: find the model owning logical tile `rem` (static kernarg indices)
    g = 0;
    int base = 0, tlg = p.tl[0];
    FDiv flg = p.fl[0];
#pragma unroll
    for (int k = 1; k < 16; ++k)
      if (k < p.G && rem >= p.tpre[k]) { g = k; base = p.tpre[k]; tlg = p.tl[k]; flg = p.fl[k]; }
    const int local = rem - base;
    if (p.cdim == 0) {  // N masked: tl[g] column tiles per row tile
      tm = (int)fdiv(local, flg);
      tn = local - tm * tlg;
    } else {            // M masked: all column tiles of tl[g] row tiles
      tm = (int)fdiv(local, p.f_tn);
      tn = local - tm * tiles_n;
    }
  } else if (p.nactive || p.nact_m || p.nact_k) {
    // masked ensembles: models carry different live sizes, so the model index varies fastest --
    // with model-major order the XCD-aware remap hands each XCD one model's tiles and the XCD
    // holding the largest model bounds the launch (measured 0.83x of unmasked at 60% live)
    g = rem % p.G;
    if (p.pair_k && ((rem >> 5) & 1)) g = p.G - 1 - g;  // (bijective: a tile row's G entries flip together)
    const int t = rem / p.G;
    tm = (int)fdiv(t, p.f_tn);
    tn = t - tm * tiles_n;
  } else {
    g = (int)fdiv(rem, p.f_plane);
    rem -= g * tiles_m * tiles_n;
    tm = (int)fdiv(rem, p.f_tn);
    tn = rem - tm * tiles_n;
  }
  const int m0 = tm * BM, n0 = tn * BN;

  // Resolve the problem's operands with selects (a dynamically indexed kernarg
  // struct would be copied to scratch).
  const bool p1 = pi != 0;
  const Operand oa0 = p1 ? p.prob[1].a[0] : p.prob[0].a[0];
  const Operand oa1 = p1 ? p.prob[1].a[1] : p.prob[0].a[1];
  const Operand ob0 = p1 ? p.prob[1].b[0] : p.prob[0].b[0];
  const Operand ob1 = p1 ? p.prob[1].b[1] : p.prob[0].b[1];
  void* cptr = p1 ? p.prob[1].c : p.prob[0].c;
  if constexpr (EPI == EPI_F32) cptr = reinterpret_cast<float*>(cptr) + ksi * p.split_stride;
  if constexpr (EPI == EPI_BF16) cptr = reinterpret_cast<uint16_t*>(cptr) + ksi * p.split_stride;
  const float alpha = p1 ? p.prob[1].alpha : p.prob[0].alpha;

  // Only the weight-gradient style epilogues take a second K segment (K-concat);
  // the fused forward epilogues never do, and skipping its offsets saves VGPRs.
  constexpr bool SEG2 = (EPI == EPI_F32 || EPI == EPI_BF16);
  constexpr bool ENC = (EPI == EPI_ENC || EPI == EPI_ENC_CNT || EPI == EPI_ENC_ACT);
  const int nk1 = p.K1 / BKT, nk_all = nk1 + (SEG2 ? p.K2 / BKT : 0);
  // this block's K-tile range [kbeg, nk) (the whole range unless split-K)
  const int kbeg = p.ksplit == 1 ? 0 : (int)fdiv(ksi * nk_all, p.f_ksplit);
  int nk = p.ksplit == 1 ? nk_all : (int)fdiv((ksi + 1) * nk_all, p.f_ksplit);
  // Masked ensembles (models with different live dictionary sizes stacked to one width,
  // reference sae_ensemble.py:306-442): output tiles wholly past a model's live columns
  // (nactive: the n dimension is N) or rows (nact_m: n is M), and K-tiles past its live
  // K range (nact_k: n is K), do no MFMA work -- the tile's epilogue still writes its zeros
  // and partial sums.  Block-uniform.
  bool dead = false;
  if (p.nactive && (ENC || EPI == EPI_DC || EPI == EPI_DC_MASK || EPI == EPI_DC_ACT)) dead = n0 >= p.nactive[g];
  if (p.nact_m) dead = dead || m0 >= p.nact_m[g];
  if (p.nact_k) nk = min(nk, (p.nact_k[g] + BKT - 1) / BKT);
  dead = dead || nk <= kbeg;
  // per-lane DMA source offsets for both K segments
  uint32_t va0[PPWA], vb0[PPWB], va1[SEG2 ? PPWA : 1], vb1[SEG2 ? PPWB : 1];
  piece_offsets<AK, BKT, PPWA>(va0, oa0.ld, m0, wid, lane);
  piece_offsets<BKM, BKT, PPWB>(vb0, ob0.ld, n0, wid, lane);
  if constexpr (SEG2) {
    piece_offsets<AK, BKT, PPWA>(va1, oa1.ld, m0, wid, lane);
    piece_offsets<BKM, BKT, PPWB>(vb1, ob1.ld, n0, wid, lane);
  }
  const i32x4_t ra0 = make_rsrc(oa0.ptr + (long)g * oa0.sg);
  const i32x4_t rb0 = make_rsrc(ob0.ptr + (long)g * ob0.sg);
  const i32x4_t ra1 = make_rsrc(oa1.ptr + (long)g * oa1.sg);
  const i32x4_t rb1 = make_rsrc(ob1.ptr + (long)g * ob1.sg);
  // soffset advance per K-tile: K-major operands step BKT elements, M/N-major BKT rows
  const uint32_t sa0 = AK ? BKT * 2 : (uint32_t)(BKT * oa0.ld * 2), sa1 = AK ? BKT * 2 : (uint32_t)(BKT * oa1.ld * 2);
  const uint32_t sb0 = BKM ? BKT * 2 : (uint32_t)(BKT * ob0.ld * 2), sb1 = BKM ? BKT * 2 : (uint32_t)(BKT * ob1.ld * 2);

#define SC_ISSUE(t)                                                              \
  do {                                                                           \
    char* dst_ = smem + ((t) % NST) * STG;                                       \
    if (!SEG2 || (t) < nk1) {                                                    \
      issue_pieces<PPWA>(ra0, va0, (uint32_t)(t) * sa0, dst_, wid);              \
      issue_pieces<PPWB>(rb0, vb0, (uint32_t)(t) * sb0, dst_ + TA, wid);         \
    } else if constexpr (SEG2) {                                                 \
      issue_pieces<PPWA>(ra1, va1, (uint32_t)((t) - nk1) * sa1, dst_, wid);      \
      issue_pieces<PPWB>(rb1, vb1, (uint32_t)((t) - nk1) * sb1, dst_ + TA, wid); \
    }                                                                            \
  } while (0)

  f32x4_t acc[WI][WJ];
#pragma unroll
  for (int i = 0; i < WI; ++i)
#pragma unroll
    for (int j = 0; j < WJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // acc[i][j][r] = C[row][col0 + r] with row = m0 + wr*16WI + i*16 + (lane&15),
  // col0 = n0 + wc*16WJ + j*16 + 4*(lane>>4).
  const int rowb = m0 + wr * (WI * 16) + (lane & 15);
  const int colb = n0 + wc * (WJ * 16) + 4 * (lane >> 4);
  // The DEC / DC epilogues read a bf16 tile of x / c at the output positions:
  // fetch it before the K loop so its HBM latency hides under the MFMAs (small
  // per-wave tiles only; at 128x64 per wave the registers are needed by the loop).
  constexpr bool AUX_EARLY = (EPI == EPI_DEC || EPI == EPI_DC || EPI == EPI_DC_ACT) && WI * WJ <= 16 && !P32;
  uint2 auxv[WI][WJ];
  if constexpr (AUX_EARLY) {
    const uint16_t* X = p.aux + (long)g * p.saux;
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
      for (int j = 0; j < WJ; ++j)
        auxv[i][j] = *reinterpret_cast<const uint2*>(X + (long)(rowb + i * 16) * p.ldaux + colb + j * 16);
  }

  // The masked code gradient's activity words (one 8-byte load per 64x64 block; 2 registers even
  // on the pipelined ring), fetched before the K loop like AUX_EARLY so their latency hides.
  uint64_t mkv[WI / 4];
  if constexpr (EPI == EPI_DC_MASK) {
#pragma unroll
    for (int k = 0; k < WI / 4; ++k)
      mkv[k] = p.cmask[mask_word(p, g, rowb - (lane & 15) + 64 * k, colb - 4 * (lane >> 4), lane)];
  }

  // The ReLU encoder epilogue's bias: loaded here, before the K-loop prologue issues its DMAs (so
  // the counted vmcnt waits below still see only tile DMAs as younger), its latency hidden.
  f32x4_t biasv[WJ];
  // (the pipelined BK32 loop needs those 16 registers: it loads the bias after the loop)
  if constexpr ((EPI == EPI_ENC || EPI == EPI_ENC_CNT) && !P32) {
    const float* bias = p.bias + (long)g * p.sbias;
#pragma unroll
    for (int j = 0; j < WJ; ++j) biasv[j] = *reinterpret_cast<const f32x4_t*>(bias + colb + j * 16);
  }

  if (!dead) {  // ---------------------------------------------------------------- K loop
#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (kbeg + t < nk) SC_ISSUE(kbeg + t);

  // Operands swapped in the MFMA (B-side rows as the MFMA's A): each lane then holds
  // 4 consecutive OUTPUT COLUMNS of one output row, so the epilogue issues 8/16-byte
  // vector stores instead of 2-byte scatters.
  auto mfmas = [&](const bf16x8_t (&fa)[WI], const bf16x8_t (&fb)[WJ]) {
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
      for (int j = 0; j < WJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
  };
  auto frags = [&](bf16x8_t (&fa)[WI], bf16x8_t (&fb)[WJ], int kt, int ks) {
    const char* la = smem + (kt % NST) * STG;
    const char* lb = la + TA;
#pragma unroll
    for (int j = 0; j < WJ; ++j) fb[j] = load_frag<BKM, BKT>(lb, wc * (WJ * 16) + j * 16, ks, lane);
#pragma unroll
    for (int i = 0; i < WI; ++i) fa[i] = load_frag<AK, BKT>(la, wr * (WI * 16) + i * 16, ks, lane);
  };

  if constexpr (BKT == 64 && S::BN == 128 && (S::BM == 128 || S::BM == 256)) {
    // Software-pipelined K loop.  The fragments of K-step s+1 are read from LDS into the
    // second register set while the MFMAs of step s run, one LDS read slotted between
    // every few MFMAs (sched_group_barrier), so no MFMA waits on an LDS round trip.  The
    // barrier of K-tile kt+1 sits before the MFMAs of tile kt's LAST step: by then every
    // wave holds tile kt entirely in registers (lgkmcnt(0)), so tile kt's stage is
    // recycled for the DMA of tile kt+NST right there, and tile kt+1's first fragment
    // reads overlap tile kt's last MFMAs.  (The accumulators use the VGPR form of the
    // MFMA -- sae_gemm.hip is built with -amdgpu-mfma-vgpr-form: with two MFMA groups per
    // iteration the AGPR form made the register allocator rotate accumulators through
    // v_accvgpr copies every iteration.)
    constexpr int RD = WI * (AK ? 1 : 2) + WJ * (BKM ? 1 : 2);  // LDS read instructions per step
    constexpr int MF = WI * WJ;                                // MFMAs per step
    constexpr int MPR = MF / RD;                               // MFMAs slotted after each read
    static_assert(MPR >= 1, "more LDS reads than MFMAs per step");
    auto step = [&](bf16x8_t (&fan)[WI], bf16x8_t (&fbn)[WJ], int ktn, int ksn, const bf16x8_t (&fa)[WI],
                    const bf16x8_t (&fb)[WJ]) {
      __builtin_amdgcn_sched_barrier(0);
      frags(fan, fbn, ktn, ksn);
      mfmas(fa, fb);
      sched_interleave<RD, MPR, MF - MPR * (RD - 1)>();
      __builtin_amdgcn_sched_barrier(0);
    };
    auto last = [&](const bf16x8_t (&fa)[WI], const bf16x8_t (&fb)[WJ]) {
      __builtin_amdgcn_sched_barrier(0);
      mfmas(fa, fb);
      __builtin_amdgcn_sched_barrier(0);
    };
    // wait until at most `younger` whole tiles of this wave's DMAs are still in flight
    auto wait_tiles = [&](int younger) {
      if (NST >= 4 && younger >= 3) wait_vmcnt<(NST >= 4 ? 3 : 0) * LPT>();
      else if (NST >= 3 && younger >= 2) wait_vmcnt<(NST >= 3 ? 2 : 0) * LPT>();
      else if (younger >= 1) wait_vmcnt<LPT>();
      else wait_vmcnt<0>();
    };
    auto tile_barrier = [&]() {
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    // the prologue above filled NST-1 stages; the last one is unused: fill it too
    if (kbeg + NST - 1 < nk) SC_ISSUE(kbeg + NST - 1);
    bf16x8_t fa0[WI], fb0[WJ], fa1[WI], fb1[WJ];
    // (the host guarantees ksplit <= number of K tiles, so every block has nk > kbeg)
    wait_tiles(min(NST - 1, nk - 1 - kbeg));  // tile kbeg landed
    tile_barrier();
    SC_STAMP(1);
    frags(fa0, fb0, kbeg, 0);
    // Steady state (a DMA issued at every boundary, NST-2 tiles younger than kt+1 in
    // flight), then the drain (no more DMAs), then the last tile peeled: neither loop body
    // branches, so the fragment and accumulator registers stay put across iterations.
    int kt = kbeg;
    for (; kt < nk - NST; ++kt) {
      step(fa1, fb1, kt, 1, fa0, fb0);
      wait_vmcnt<(NST - 2) * LPT>();  // tile kt+1 landed; kt+2 .. kt+NST-1 may be in flight
      tile_barrier();
      SC_ISSUE(kt + NST);
      step(fa0, fb0, kt + 1, 0, fa1, fb1);
    }
    for (; kt < nk - 1; ++kt) {
      step(fa1, fb1, kt, 1, fa0, fb0);
      wait_tiles(min(NST - 2, nk - 2 - kt));
      tile_barrier();
      step(fa0, fb0, kt + 1, 0, fa1, fb1);
    }
    step(fa1, fb1, nk - 1, 1, fa0, fb0);
    last(fa1, fb1);
  } else if constexpr (P32 && BKT == 32 && S::BM == 128 && S::BN == 128) {
    // The same software pipeline for the BK32 rings (one 32-deep MFMA step per K-tile, 48 KB at
    // three stages: three workgroups per CU): tile kt+1's fragments are read into the second
    // register set while tile kt's MFMAs run.  At the barrier before those reads every wave holds
    // tile kt in registers (lgkmcnt(0)), so tile kt's stage takes the DMA of tile kt+NST there.
    // Unrolled by two for the register ping-pong; steady state (a DMA at both barriers), drain,
    // last tile.
    constexpr int RD = WI * (AK ? 1 : 2) + WJ * (BKM ? 1 : 2);
    constexpr int MF = WI * WJ;
    constexpr int MPR = MF / RD;
    static_assert(MPR >= 1, "more LDS reads than MFMAs per step");
    auto step = [&](bf16x8_t (&fan)[WI], bf16x8_t (&fbn)[WJ], int ktn, const bf16x8_t (&fa)[WI],
                    const bf16x8_t (&fb)[WJ]) {
      __builtin_amdgcn_sched_barrier(0);
      frags(fan, fbn, ktn, 0);
      mfmas(fa, fb);
      sched_interleave<RD, MPR, MF - MPR * (RD - 1)>();
      __builtin_amdgcn_sched_barrier(0);
    };
    auto last = [&](const bf16x8_t (&fa)[WI], const bf16x8_t (&fb)[WJ]) {
      __builtin_amdgcn_sched_barrier(0);
      mfmas(fa, fb);
      __builtin_amdgcn_sched_barrier(0);
    };
    auto wait_tiles = [&](int younger) {
      if (NST >= 4 && younger >= 3) wait_vmcnt<(NST >= 4 ? 3 : 0) * LPT>();
      else if (NST >= 3 && younger >= 2) wait_vmcnt<(NST >= 3 ? 2 : 0) * LPT>();
      else if (younger >= 1) wait_vmcnt<LPT>();
      else wait_vmcnt<0>();
    };
    auto tile_barrier = [&]() {
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    if (kbeg + NST - 1 < nk) SC_ISSUE(kbeg + NST - 1);  // all NST stages in flight
    bf16x8_t fa0[WI], fb0[WJ], fa1[WI], fb1[WJ];
    wait_tiles(min(NST - 1, nk - 1 - kbeg));  // tile kbeg landed
    tile_barrier();
    SC_STAMP(1);
    frags(fa0, fb0, kbeg, 0);
    int kt = kbeg;  // invariant: fa0 / fb0 hold tile kt
    for (; kt + 1 + NST < nk; kt += 2) {
      wait_vmcnt<(NST - 2) * LPT>();  // tile kt+1 landed
      tile_barrier();
      SC_ISSUE(kt + NST);
      step(fa1, fb1, kt + 1, fa0, fb0);
      wait_vmcnt<(NST - 2) * LPT>();  // tile kt+2 landed
      tile_barrier();
      SC_ISSUE(kt + 1 + NST);
      step(fa0, fb0, kt + 2, fa1, fb1);
    }
    for (; kt + 2 < nk; kt += 2) {
      wait_tiles(min(NST - 2, nk - 2 - kt));
      tile_barrier();
      if (kt + NST < nk) SC_ISSUE(kt + NST);
      step(fa1, fb1, kt + 1, fa0, fb0);
      wait_tiles(min(NST - 2, nk - 3 - kt));
      tile_barrier();
      step(fa0, fb0, kt + 2, fa1, fb1);
    }
    if (kt + 1 < nk) {
      wait_tiles(0);
      tile_barrier();
      step(fa1, fb1, kt + 1, fa0, fb0);
      last(fa1, fb1);
    } else {
      last(fa0, fb0);
    }
  } else for (int kt = kbeg; kt < nk; ++kt) {
    // Tile kt must have landed; tiles kt+1 .. kt+NST-2 may stay in flight.
    const int younger = min(NST - 2, nk - 1 - kt);
    if constexpr (NST >= 4) {
      if (younger >= 2) wait_vmcnt<2 * LPT>();
      else if (younger == 1) wait_vmcnt<LPT>();
      else wait_vmcnt<0>();
    } else if constexpr (NST == 3) {
      if (younger >= 1) wait_vmcnt<LPT>();
      else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    // lgkmcnt(0): this wave's reads of the stage being recycled are done; raw barrier
    // (no implicit vmcnt(0)) so younger DMAs stay in flight; "memory" keeps hipcc from
    // moving LDS reads across it.
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt == kbeg) SC_STAMP(1);
    if (kt + NST - 1 < nk) SC_ISSUE(kt + NST - 1);
    const char* la = smem + (kt % NST) * STG;
    const char* lb = la + TA;
#pragma unroll
    for (int ks = 0; ks < BKT / 32; ++ks) {
      bf16x8_t fa[WI], fb[WJ];
#pragma unroll
      for (int j = 0; j < WJ; ++j) fb[j] = load_frag<BKM, BKT>(lb, wc * (WJ * 16) + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < WI; ++i) fa[i] = load_frag<AK, BKT>(la, wr * (WI * 16) + i * 16, ks, lane);
      // Operands swapped (B-side rows as the MFMA's A): each lane then holds
      // 4 consecutive OUTPUT COLUMNS of one output row, so the epilogue
      // issues 8/16-byte vector stores instead of 2-byte scatters.
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int j = 0; j < WJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  }  // !dead
#undef SC_ISSUE
  SC_STAMP(2);
  if constexpr ((EPI == EPI_ENC || EPI == EPI_ENC_CNT) && P32) {
    const float* bias = p.bias + (long)g * p.sbias;
#pragma unroll
    for (int j = 0; j < WJ; ++j) biasv[j] = *reinterpret_cast<const f32x4_t*>(bias + colb + j * 16);
  }
  lds_barrier();  // all reads of the ring done before smem is reused below
  SC_SUB(6);
  constexpr bool STAGE = (S::WI == 4 || S::WI == 8) && S::WJ == 4 && NST * STG >= stage_bytes<S>();
  constexpr bool FSTAGE = EPI == EPI_F32 && S::WJ == 4 && NST * STG >= S::NW * S::WI * 16 * STAGE_ROW;
  sae_epilogue<S, EPI, AUX_EARLY, STAGE, FSTAGE>(p, acc, auxv, biasv, mkv, reinterpret_cast<float*>(smem), pi, g, m0, n0, tn,
                                                 tiles_n, cptr, alpha, dead);
  SC_STAMP(3);
}

// (the software-pipelined BK32 x 3 loop: three waves per SIMD, so three blocks co-reside per CU)
template <class S, bool AK, bool BKM, int EPI, int BKT, int NST, bool P32 = false>
// (the eight-wave 256x128 block on BK32 x 3: four waves per SIMD, i.e. two blocks per CU -- the second
// launch-bounds argument is waves per execution unit)
__global__ __launch_bounds__(S::NT, (P32 && NST == 3) ? 3 : ((S::NW == 8 && S::BN == 128 && NST == 3) ? 4 : 1)) void sae_gemm_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[NST * (S::BM + S::BN) * BKT * 2];
  gemm_block<S, AK, BKM, EPI, BKT, NST, P32>(p, xcd_remap(blockIdx.x, gridDim.x), smem);
}


}  // namespace scamd

namespace scamd {
template <class S>
bool fits(int M, int N) { return M % S::BM == 0 && N % S::BN == 0; }

template <class S>
long n_blocks(int M, int N, int G, int nprob) { return (long)(M / S::BM) * (N / S::BN) * G * nprob; }

// FULL = every (layout, epilogue) pair; the alternative K pipelines (deeper LDS rings,
// selected with cfg bits 2-3) instantiate only the step's epilogues and the weight-gradient
// layout, to keep the build small.
// Host: the decomposition divisors for block shape S (ksplit-aware).
template <class S>
void set_divisors(GemmParams& p) {
  const uint32_t tn = p.N / S::BN, plane = (uint32_t)(p.M / S::BM) * tn, split = plane * p.G;
  p.f_tn = make_fdiv(tn);
  p.f_plane = make_fdiv(plane);
  p.f_split = make_fdiv(split);
  p.f_prob = make_fdiv(split * p.ksplit);
  p.f_ksplit = make_fdiv(p.ksplit);
}

// Host: compact a masked launch to its live tiles (see GemmParams::ncomp).  Returns the number of
// blocks per problem, or 0 when the launch stays uncompacted.
template <class S>
long compact_tiles(int epi, GemmParams& p) {
  p.ncomp = 0;
  if (!p.want_comp || p.G > 16) return 0;
  const bool ncols = p.nactive && (epi == EPI_ENC || epi == EPI_ENC_CNT || epi == EPI_ENC_ACT || epi == EPI_DC ||
                                   epi == EPI_DC_MASK || epi == EPI_DC_ACT);
  const bool nrows = p.nact_m && (epi == EPI_F32 || epi == EPI_BF16);
  if (!ncols && !nrows) return 0;
  const int per = ncols ? S::BN : S::BM, full = ncols ? p.N / S::BN : p.M / S::BM;
  const int other = ncols ? p.M / S::BM : p.N / S::BN;
  long total = 0;
  for (int g = 0; g < p.G; ++g) {
    const int live = std::min(full, std::max(1, (p.nact_h[g] + per - 1) / per));
    p.tl[g] = live;
    p.fl[g] = make_fdiv((uint32_t)live);
    p.tpre[g] = (int)total;
    total += (long)live * other;
  }
  p.tpre[p.G] = (int)total;
  p.ctotal = (int)total;
  p.ncomp = 1;
  p.cdim = ncols ? 0 : 1;
  return total;
}

// Host: the masked decoder's block pairing.  Its per-model K range (live size) sets each tile's cost,
// and a CU's two co-resident tiles share its operand feed, so a CU is busy for about the SUM of its
// tiles' K ranges.  The hardware places blocks j and j + 32 of one XCD's dispatch sequence (j = blockIdx
// / 8) on the same CU (per-block HW_ID stamps, profiles/r5/batch28/); with the model index varying
// fastest both carried the same model, so the CUs holding the largest model paired two full-K tiles and
// set the launch.  Flipping the model index of every second run of 32 logical tiles (g -> G-1-g) pairs
// g with G-1-g instead: every CU then carries about the mean K range.  Needs the XCD runs of xcd_remap
// to start on multiples of 32 and G | 32; otherwise the order is unchanged.
// (Measured -1.1 % on the masked step, profiles/r5/batch29/; the A/B switch is gone -- always on.)
inline int pair_order(const GemmParams& p, long comp, long nwg, int nprob) {
  return !comp && p.nact_k && !p.nactive && !p.nact_m && p.ksplit == 1 && nprob == 1 && p.G >= 2 &&
         32 % p.G == 0 && nwg % 256 == 0;
}

template <class S, int BKT, int NST, bool FULL = true, bool P32 = false>
int launch(int epi, bool ak, bool bk, GemmParams p, int nprob, hipStream_t stream) {
  set_divisors<S>(p);
  const long comp = compact_tiles<S>(epi, p);
  if (comp) {
    p.f_split = make_fdiv((uint32_t)comp);
    p.f_prob = make_fdiv((uint32_t)(comp * p.ksplit));
  }
  const dim3 grid((unsigned)((comp ? comp * nprob : n_blocks<S>(p.M, p.N, p.G, nprob)) * p.ksplit)), block(S::NT);
  p.pair_k = pair_order(p, comp, grid.x, nprob);
  if constexpr (!FULL) {
    // (the BK32 rings: the fused step epilogues, the fp32 weight-gradient layout and the bf16 plain
    // epilogue in the top-k layouts -- scores x D^T, codes^T R)
    if (epi >= EPI_ENC_ACT || (epi == EPI_F32 && (ak || bk)) || (epi == EPI_BF16 && ak != bk)) return 8;
  }
#define SC_L(AKV, BKV, E) hipLaunchKernelGGL((sae_gemm_kernel<S, AKV, BKV, E, BKT, NST, P32>), grid, block, 0, stream, p)
  // Only the (layout, epilogue) pairs the engine uses are instantiated for the fused
  // epilogues; the plain F32 / BF16 epilogues exist for every layout.
  switch (epi) {
    case EPI_ENC: if (!(ak && bk)) return 5; SC_L(true, true, EPI_ENC); break;
    case EPI_ENC_CNT: if (!(ak && bk)) return 5; SC_L(true, true, EPI_ENC_CNT); break;
    case EPI_DEC: if (!(ak && !bk)) return 5; SC_L(true, false, EPI_DEC); break;
    case EPI_DC: if (!(ak && bk)) return 5; SC_L(true, true, EPI_DC); break;
    case EPI_DC_MASK: if (!(ak && bk)) return 5; SC_L(true, true, EPI_DC_MASK); break;
    case EPI_ENC_ACT:
      if constexpr (FULL) { if (!(ak && bk)) return 5; SC_L(true, true, EPI_ENC_ACT); }
      break;
    case EPI_DC_ACT:
      if constexpr (FULL) { if (!(ak && bk)) return 5; SC_L(true, true, EPI_DC_ACT); }
      break;
    case EPI_ROWMAX:
      if constexpr (FULL) { if (!(ak && bk)) return 5; SC_L(true, true, EPI_ROWMAX); }
      break;
    case EPI_F32:
      if constexpr (FULL) {
        if (ak && bk) SC_L(true, true, EPI_F32);
        else if (ak) SC_L(true, false, EPI_F32);
        else if (bk) SC_L(false, true, EPI_F32);
        else SC_L(false, false, EPI_F32);
      } else {
        SC_L(false, false, EPI_F32);
      }
      break;
    case EPI_BF16:
      if constexpr (FULL) {
        if (ak && bk) SC_L(true, true, EPI_BF16);
        else if (ak) SC_L(true, false, EPI_BF16);
        else if (bk) SC_L(false, true, EPI_BF16);
        else SC_L(false, false, EPI_BF16);
      } else {
        if (ak) SC_L(true, true, EPI_BF16);
        else SC_L(false, false, EPI_BF16);
      }
      break;
    default: return 2;
  }
#undef SC_L
  return hipGetLastError() == hipSuccess ? 0 : 3;
}


// 256x128 / 256x256 launches (sae_gemm_big.hip)
int launch_big(int shape, int pipe, int epi, bool ak, bool bk, const GemmParams& p, int nprob, hipStream_t stream);
int launch_256x128(int pipe, int epi, bool ak, bool bk, const GemmParams& p, int nprob, hipStream_t stream);

}  // namespace scamd
