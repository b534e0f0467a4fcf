// Row-block fused SAE forward + code gradient (gfx950): the encoder, decoder and code-gradient
// GEMMs of one training step in ONE launch.
//
// The separate kernels (sae_gemm_kernel.h: EPI_ENC -> EPI_DEC -> EPI_DC_MASK) each pay a
// prologue (first operand tiles in flight), an un-overlapped epilogue store tail, and a re-read
// of the previous kernel's output from HBM/MALL (c for the decoder, R for the code gradient).
// Here one workgroup owns 64 batch rows of one model and streams that model's dictionaries
// through LDS three times:
//
//   phase A, per 256-feature chunk j:   c_j = relu(x We_j^T + b_j)   (K = d, A = x slices)
//                                       R  += c_j W_hat_j            (c_j stays in LDS)
//   end of A:                           R  -= x  -> bf16 R to HBM, sum R^2
//   phase C, per chunk j:               dpre_j = 1[c_j > 0] (R W_hat_j^T + l1 d/2)
//
// so c never round-trips for the decoder and R only once (L2-hot) for the code gradient; the
// c / R / dpre stores (needed by the weight-gradient GEMM) drain under the next chunk's MFMAs.
// Reference math: autoencoders/sae_ensemble.py:53-77 (FunctionalSAE.loss) and its autograd
// (SURVEY Appendix A); gradients are in units of 2/(B d) exactly as the separate epilogues.
//
// Layout: 512 threads = 8 waves (2 per SIMD, 1 workgroup per CU), waves as 2 row groups (32 rows)
// x 4 column groups.  v_mfma_f32_16x16x32_bf16 with the operands swapped (lane = 4 consecutive
// output columns of one row, as in sae_gemm_kernel.h).  The three dictionary streams are one
// sequence of LDS-DMA "units" through a 6-slot ring of 21 KiB:
//   enc unit: We_j[256 rows][32 k] (16 KiB, K-major) + x[64 rows][32 k] (4 KiB)
//   dec unit: W_hat_j[32 k-rows][256 cols] (16 KiB, N-major: transposing ds_read_b64_tr_b16)
//   dc  unit: W_hat_j[256 rows][32 k] + R[64 rows][32 k] (R read back from L2)
// one barrier per PAIR of units, the four units after the pair in flight while it computes.
// Grid: G * B/64 workgroups, XCD-remapped so each XCD serves one model (its dictionaries stay in
// that XCD's L2 while 32 CUs stream them).
#include "gemm_tiles.h"


namespace scamd {

struct RowBlockParams {
  const uint16_t* x;  // [G?][B][D] bf16 (x_sg = 0: one batch shared by every model)
  long x_sg;
  const uint16_t* we;  // [G][n][D] encoder bf16 shadow
  const uint16_t* wd;  // [G][n][D] row-normalised decoder bf16 shadow
  const float* bias;   // [G][n]
  const float* l1;     // [G]
  float l1_add;        // d / 2: dpre in units of R
  uint16_t* c;         // [G][B][n]
  uint16_t* r;         // [G][B][D]
  uint16_t* dpre;      // [G][B][n]
  uint32_t* cmask;     // activity bitmask (sae_gemm_kernel.h mask_word layout, as 32-bit halves)
  float* enc_part;     // [G][B/64][2]  (sum |c|, number of active codes)
  float* dec_part;     // [G][B/64]     (sum R^2)
  float* colpart;      // [G][B/32][n]  bias-gradient partial sums (32-row slots)
  float* cnt_part;     // [G][B/32][n]  feature on-counts (null: not counted this step)
  int G, B, n;
};

// Per-step timestamps of one workgroup (lab builds only: scripts/lab/rowblock_stamps.hip defines
// SC_RB_STAMPS; product builds compile these to nothing).  Slot k of step b of wave w:
// 0 step start, 1 own DMAs landed, 2 barrier passed, 3 compute done.
#ifdef SC_RB_STAMPS
__device__ long long* sc_rb_stamps;
__device__ int sc_rb_block;
#define RB_STAMP(b, k)                                                                 \
  do {                                                                                 \
    if (rb_st && lane == 0) rb_st[((long)wid * 1024 + (b)) * 4 + (k)] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
#define RB_STAMP_INIT long long* const rb_st = (int)blockIdx.x == sc_rb_block ? sc_rb_stamps : nullptr
#else
#define RB_STAMP(b, k) do {} while (0)
#define RB_STAMP_INIT do {} while (0)
#endif

namespace rb {
constexpr int D = 512, BR = 64, NC = 256, NT = 512, NW = 8;
constexpr int C_BYTES = BR * NC * 2;           // 32 KiB: c_j / dpre_j as 8 K-major [64][32] slices
// Ring of NSLOT unit slots: B part (16 KiB), A part (4 KiB), and the chunk's encoder bias (1 KiB,
// last encoder unit of each chunk: the epilogue reads it from LDS, so no global load inside the
// loop makes the compiler drain the DMA pipeline with a vmcnt(0)).  Five units stay in flight
// behind the one being consumed: the stream is latency-bound otherwise (one 40 KiB unit of
// lookahead measured 230 us for the three phases).
constexpr int SLOT = 21504, SLOT_A = 16384, SLOT_BIAS = 20480;
constexpr int RING = C_BYTES, NSLOT = 6;
constexpr int SCRATCH = RING + NSLOT * SLOT;   // 161792
constexpr int MAXCH = 8;                       // n <= 2048: activity words of every chunk in registers
constexpr int LDS_BYTES = SCRATCH + 64;
static_assert(LDS_BYTES <= 163840, "LDS budget");
constexpr int UPC_A = 32, UPC_C = 16;          // units per chunk: phase A (16 enc + 16 dec), phase C

// byte offset of the 8-byte group holding columns c..c+3 (c % 4 == 0) of row `row` in the
// [64][256] bf16 image made of 8 K-major [64][32] slices (kmaj_off<32>)
__device__ __forceinline__ int cimg_off(int row, int c) {
  return (c >> 5) * 4096 + kmaj_off<32>(row, (c & 31) >> 3) + ((c >> 2) & 1) * 8;
}

}  // namespace rb

template <bool COUNT>
__global__ __launch_bounds__(rb::NT) void sae_rowblock_kernel(RowBlockParams p) {
  using namespace rb;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  char* const cimg = smem;
  RB_STAMP_INIT;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int nrb = p.B / BR;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int g = L / nrb, rbk = L - g * nrb;
  const int m0 = rbk * BR;
  const int n = p.n, nch = n / NC;
  const int UA = UPC_A * nch, U = UA + UPC_C * nch;  // phase-A units, all units

  // Unit sequence (one barrier each):
  //   phase A, chunk j:  w = 0..15   enc: We_j[256][32 k of slice w] + x[64][32 k]      (K-major)
  //                      w = 16..31  dec: W_hat_j[32 k-rows t = (w-16)/2][256 cols h = w&1] (N-major)
  //   phase C, chunk j:  s = 0..15   dc:  W_hat_j[256][32 k of slice s] + R[64][32 k]  (K-major)
  // per-lane LDS-DMA source offsets are unit-invariant; the unit adds a scalar soffset
  // Only waves 0-3 (one per SIMD) issue DMAs: the per-piece scalar bookkeeping runs on the CU's
  // single scalar unit, and with all 8 waves issuing the loop was scalar-issue bound.
  const bool dma_wave = wid < 4;
  uint32_t vB[4], vA[1], vT[4];
  piece_offsets<true, 32, 4>(vB, D, 0, wid & 3, lane);           // [256 rows][32 k]: 16 pieces
  piece_offsets<true, 32, 1>(vA, D, m0, wid & 3, lane);          // [64 rows][32 k]: 4 pieces
  piece_offsets<false, 32, 4>(vT, D, 0, wid & 3, lane);          // [32 k][256 cols]: 16 pieces
  const i32x4_t rWe = make_rsrc(p.we + (long)g * n * D);
  const i32x4_t rWd = make_rsrc(p.wd + (long)g * n * D);
  const i32x4_t rX = make_rsrc(p.x + (long)g * p.x_sg);
  const i32x4_t rR = make_rsrc(p.r + (long)g * p.B * D);
  const i32x4_t rBias = make_rsrc(reinterpret_cast<const uint16_t*>(p.bias + (long)g * n));
  const uint32_t vBias = (uint32_t)lane * 16u;

  // The scalar unit is shared by the CU's 8 waves and every wave runs this bookkeeping, so the
  // per-unit scalar path is kept to a few dozen instructions (a first version that decoded each
  // unit from scratch and summed per-unit DMA counts for the wait was scalar-issue bound:
  // ~350 us with no DMA and no MFMA at all).
  auto issue = [&](int u, int slotk) {
    char* slot = smem + RING + slotk * SLOT;
    if (u < UA) {
      const int j = u >> 5, w = u & 31;
      if (w < 16) {
        issue_pieces<4>(rWe, vB, (uint32_t)(j * NC * D + 32 * w) * 2u, slot, wid);
        issue_pieces<1>(rX, vA, (uint32_t)(32 * w) * 2u, slot + SLOT_A, wid);
        if (w == 15 && wid == 0) issue_pieces<1>(rBias, &vBias, (uint32_t)(j * NC * 4), slot + SLOT_BIAS, 0);
      } else {
        const int t = (w - 16) >> 1, h = w & 1;
        issue_pieces<4>(rWd, vT, (uint32_t)((j * NC + 32 * t) * D + 256 * h) * 2u, slot, wid);
      }
    } else {
      const int v = u - UA, j = v >> 4, sl = v & 15;
      issue_pieces<4>(rWd, vB, (uint32_t)(j * NC * D + 32 * sl) * 2u, slot, wid);
      issue_pieces<1>(rR, vA, (uint32_t)(32 * sl) * 2u, slot + SLOT_A, wid);
    }
  };

  f32x4_t acc_r[2][8];  // R rows 32wr + 16i, columns 256 (jd >> 2) + 64wc + 16 (jd & 3)
  f32x4_t acc[2][4];    // c_j / dpre_j rows 32wr + 16i, columns 64wc + 16jj
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc_r[i][k] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[i][k] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  float l1s = 0.f, l0s = 0.f, se = 0.f;
  const float add = p.l1[g] * p.l1_add;
  const long slot32 = (long)g * (p.B / 32) + 2 * rbk + wr;  // 32-row partial slot of this wave
  // mask word (64x64 block at rows m0, columns col0) of this lane, as the 32-bit half of wave row wr
  auto mask_at = [&](int col0) -> uint32_t* {
    return p.cmask + ((((long)g * nrb + rbk) * (n >> 6) + (col0 >> 6)) * 64 + lane) * 2 + wr;
  };

  // stores of the [64][256] bf16 image in cimg to out[row][col0 ..] (row stride n), all threads
  auto store_cimg = [&](uint16_t* out, int col0) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int q = tid + it * NT, row = q >> 5, ch32 = q & 31;
      const uint4 v = *reinterpret_cast<const uint4*>(cimg + (ch32 >> 2) * 4096 + kmaj_off<32>(row, ch32 & 3));
      *reinterpret_cast<uint4*>(out + ((long)g * p.B + m0 + row) * n + col0 + ch32 * 8) = v;
    }
  };

  // one K-major k-step on a [256][32] B slice and a [64][32] A slice: acc += A B^T
  auto kstep = [&](const char* slot) {
    bf16x8_t fa[2], fb[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) fb[jj] = load_frag<true, 32>(slot, 64 * wc + 16 * jj, 0, lane);
#pragma unroll
    for (int i = 0; i < 2; ++i) fa[i] = load_frag<true, 32>(slot + SLOT_A, 32 * wr + 16 * i, 0, lane);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[jj], fa[i], acc[i][jj], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // decoder k-step t on both column halves of R: acc_r += c_j[:, 32t..] W_hat_j[32t.., :]
  // (slot0: columns 0..255, slot1: 256..511; the c fragments are read once for both)
  auto dstep2 = [&](const char* slot0, const char* slot1, int t) {
    bf16x8_t fa[2], fb[4], fb1[4];
#pragma unroll
    for (int i = 0; i < 2; ++i) fa[i] = load_frag<true, 32>(cimg + t * 4096, 32 * wr + 16 * i, 0, lane);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) fb[jj] = load_frag<false, 32>(slot0, 64 * wc + 16 * jj, 0, lane);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) fb1[jj] = load_frag<false, 32>(slot1, 64 * wc + 16 * jj, 0, lane);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        acc_r[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[jj], fa[i], acc_r[i][jj], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        acc_r[i][4 + jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[jj], fa[i], acc_r[i][4 + jj], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // activity words of this lane, one per chunk, as a FIFO with static register indices (a
  // dynamically indexed array would live in scratch): phase A shifts each chunk's word in at
  // the top, phase C aligns chunk 0 to slot 0 and shifts one out per chunk
  uint32_t mq[MAXCH];
#pragma unroll
  for (int k = 0; k < MAXCH; ++k) mq[k] = 0u;
  auto mq_shift = [&](uint32_t in) {
#pragma unroll
    for (int k = 0; k < MAXCH - 1; ++k) mq[k] = mq[k + 1];
    mq[MAXCH - 1] = in;
  };

  int issued = 0, islot = 0, limit = UA;
  auto refill = [&](int upto) {  // issue units up to `upto` (inclusive) within the phase limit
    while (issued <= upto && issued < limit) {
      if (dma_wave) issue(issued, islot);
      ++issued;
      islot = islot == NSLOT - 1 ? 0 : islot + 1;
    }
  };
  // Units are consumed in PAIRS, one barrier per pair (a single unit is only 8 MFMAs per wave:
  // barrier, LDS latency and DMA issue dominated at one barrier per unit); the NSLOT-2 units
  // after the pair stay in flight.  Pairs never straddle a phase (16 units per chunk and part).
  refill(NSLOT - 3);
  int cslot = 0;  // ring slot of unit b (even)
  for (int b = 0; b < U; b += 2) {
    if (b == UA) {
      // ---- end of phase A: R = acc_r - x -> bf16 to HBM (the dc units read it back), sum R^2
      // all 16 x loads first (the stores below may alias x for the compiler, which would
      // otherwise serialise every load behind the previous store: 16 round trips)
      const uint16_t* X = p.x + (long)g * p.x_sg;
      uint2 xr[2][8];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jd = 0; jd < 8; ++jd)
          xr[i][jd] = *reinterpret_cast<const uint2*>(X + (long)(m0 + 32 * wr + 16 * i + (lane & 15)) * D +
                                                      256 * (jd >> 2) + 64 * wc + 16 * (jd & 3) + 4 * (lane >> 4));
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const long row = m0 + 32 * wr + 16 * i + (lane & 15);
#pragma unroll
        for (int jd = 0; jd < 8; ++jd) {
          const int col = 256 * (jd >> 2) + 64 * wc + 16 * (jd & 3) + 4 * (lane >> 4);
          const uint2 xv = xr[i][jd];
          const float r0 = acc_r[i][jd][0] - bf2f(xv.x & 0xFFFF), r1 = acc_r[i][jd][1] - bf2f(xv.x >> 16);
          const float r2 = acc_r[i][jd][2] - bf2f(xv.y & 0xFFFF), r3 = acc_r[i][jd][3] - bf2f(xv.y >> 16);
          se += r0 * r0 + r1 * r1 + r2 * r2 + r3 * r3;
          *reinterpret_cast<ushort4*>(p.r + ((long)g * p.B + row) * D + col) =
              make_ushort4(f2bf(r0), f2bf(r1), f2bf(r2), f2bf(r3));
        }
      }
      // every wave's R stores complete before any wave's DMA reads them back
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      for (int k = nch; k < MAXCH; ++k) mq_shift(0u);  // chunk 0's word to mq[0]
      limit = U;
      refill(b + NSLOT - 3);
    }
    RB_STAMP(b, 0);
    // Units b, b+1 must have landed (the DMA waves wait for their own pieces; the barrier then
    // publishes them to all).  Every unit puts >= 4 DMA instructions per DMA wave in flight, so
    // with the two younger units issued vmcnt(8) is a safe (slightly conservative) bound.
    if (dma_wave) {
      if (issued - 2 - b >= 2) wait_vmcnt<8>();
      else wait_vmcnt<0>();
    }
    RB_STAMP(b, 1);
    lds_barrier();
    RB_STAMP(b, 2);
    refill(b + NSLOT - 1);
    const char* slot0 = smem + RING + cslot * SLOT;
    const char* slot1 = slot0 + SLOT;
    cslot = cslot == NSLOT - 2 ? 0 : cslot + 2;

    if (b < UA) {
      const int j = b >> 5, w = b & 31;
      if (w < 16) {
        // ---------------- encoder: acc += x_slice We_slice^T (two K-slices)
        kstep(slot0);
        kstep(slot1);
        if (w == 14) {
          // c_j = relu(acc + b): bf16 image for the decoder (and the HBM store), bitmask, L1/L0
          const int colb = j * NC + 64 * wc + 4 * (lane >> 4);
          uint32_t mw = 0;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const f32x4_t bj = *reinterpret_cast<const f32x4_t*>(slot1 + SLOT_BIAS + (64 * wc + 16 * jj + 4 * (lane >> 4)) * 4);
            f32x4_t cnt = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 2; ++i) {
              f32x4_t v;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                v[r] = fmaxf(acc[i][jj][r] + bj[r], 0.f);
                l1s += v[r];
                const bool on = v[r] > 0.f;
                mw |= on ? (1u << ((i * 4 + jj) * 4 + r)) : 0u;
                if (COUNT) cnt[r] += on ? 1.f : 0.f;
              }
              *reinterpret_cast<ushort4*>(cimg + cimg_off(32 * wr + 16 * i + (lane & 15), 64 * wc + 16 * jj + 4 * (lane >> 4))) =
                  make_ushort4(f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3]));
              acc[i][jj] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            }
            if (COUNT) {
#pragma unroll
              for (int r = 0; r < 4; ++r) cnt[r] = row16_scan(cnt[r]);
              if ((lane & 15) == 15) *reinterpret_cast<f32x4_t*>(p.cnt_part + slot32 * n + colb + 16 * jj) = cnt;
            }
          }
          *mask_at(j * NC + 64 * wc) = mw;
          mq_shift(mw);
          l0s += (float)__popc(mw);
        }
      } else {
        // ---------------- decoder: R += c_j[:, 32t..] W_hat_j[32t.., :] (both column halves)
        const int t = (w - 16) >> 1;
        if (w == 16) store_cimg(p.c, j * NC);  // c_j image complete (barrier above): to HBM
        dstep2(slot0, slot1, t);
      }
    } else {
      // ---------------- code gradient: acc += R_slice W_hat_slice^T (two K-slices)
      const int v = b - UA, j = v >> 4, s = v & 15;
      if (s == 0 && j > 0) store_cimg(p.dpre, (j - 1) * NC);  // previous chunk's dpre image
      kstep(slot0);
      kstep(slot1);
      if (s == 14) {
        const uint32_t mk = mq[0];
        mq_shift(0u);
        const int colb = j * NC + 64 * wc + 4 * (lane >> 4);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          f32x4_t cs = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            f32x4_t dv;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const bool on = (mk >> ((i * 4 + jj) * 4 + r)) & 1u;
              dv[r] = on ? acc[i][jj][r] + add : 0.f;
              cs[r] += dv[r];
            }
            *reinterpret_cast<ushort4*>(cimg + cimg_off(32 * wr + 16 * i + (lane & 15), 64 * wc + 16 * jj + 4 * (lane >> 4))) =
                make_ushort4(f2bf(dv[0]), f2bf(dv[1]), f2bf(dv[2]), f2bf(dv[3]));
            acc[i][jj] = f32x4_t{0.f, 0.f, 0.f, 0.f};
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) cs[r] = row16_scan(cs[r]);
          if ((lane & 15) == 15) *reinterpret_cast<f32x4_t*>(p.colpart + slot32 * n + colb + 16 * jj) = cs;
        }
      }
    }
    RB_STAMP(b, 3);
  }
  lds_barrier();
  store_cimg(p.dpre, (nch - 1) * NC);
  float* red = reinterpret_cast<float*>(smem + SCRATCH);
  l1s = block_sum_lds<NW>(l1s, red);
  l0s = block_sum_lds<NW>(l0s, red);
  se = block_sum_lds<NW>(se, red);
  if (tid == 0) {
    const long o = (long)g * nrb + rbk;
    p.enc_part[o * 2] = l1s;
    p.enc_part[o * 2 + 1] = l0s;
    p.dec_part[o] = se;
  }
}

}  // namespace scamd

extern "C" {

// Shapes: d == 512, n % 256 == 0, n <= 2048, B % 64 == 0.  Returns 0 on success, 1 on unsupported shape,
// 3 on launch error.
int sc_sae_rowblock(const void* x, long x_sg, const void* we, const void* wd, const void* bias, const void* l1,
                    float l1_add, void* c, void* r, void* dpre, void* cmask, void* enc_part, void* dec_part,
                    void* colpart, void* cnt_part, int G, int B, int n, int d, hipStream_t stream) {
  using namespace scamd;
  if (d != rb::D || n % rb::NC || n <= 0 || n > rb::MAXCH * rb::NC || B % rb::BR || B <= 0 || G <= 0) return 1;
  RowBlockParams p;
  p.x = (const uint16_t*)x; p.x_sg = x_sg;
  p.we = (const uint16_t*)we; p.wd = (const uint16_t*)wd;
  p.bias = (const float*)bias; p.l1 = (const float*)l1; p.l1_add = l1_add;
  p.c = (uint16_t*)c; p.r = (uint16_t*)r; p.dpre = (uint16_t*)dpre; p.cmask = (uint32_t*)cmask;
  p.enc_part = (float*)enc_part; p.dec_part = (float*)dec_part;
  p.colpart = (float*)colpart; p.cnt_part = (float*)cnt_part;
  p.G = G; p.B = B; p.n = n;
  const dim3 grid((unsigned)(G * (B / rb::BR))), block(rb::NT);
  if (cnt_part) hipLaunchKernelGGL(sae_rowblock_kernel<true>, grid, block, 0, stream, p);
  else hipLaunchKernelGGL(sae_rowblock_kernel<false>, grid, block, 0, stream, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
