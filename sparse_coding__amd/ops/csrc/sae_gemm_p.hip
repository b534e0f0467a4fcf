// Persistent, wave-specialised grouped bf16 MFMA GEMM with fused SAE epilogues (gfx950).
//
// The step GEMMs of an SAE ensemble are short-K with large bf16 outputs: the encoder
// (c = relu(x W_e^T + b), K = d = 512) and the code gradient (dpre = mask (R W_hat^T + l),
// K = d) write G x B x n bf16 values after only 512 MACs each.  Per output element the MFMA
// work is ~1 SIMD-cycle and the epilogue (bias / ReLU / L1-L0 statistics / activity ballots /
// a 2-byte store) costs about as much again, so a tile kernel that runs "main loop, then
// epilogue" leaves the matrix cores idle for a large share of the time (MI355X, G=8,
// B=n=2048: the plain bf16 GEMM takes 26 us at K=64 and 48 us at K=512 -- the fixed per-tile
// cost is half the kernel; profiles/gemm_lab_r2_v1.jsonl).
//
// Structure (reference math: autoencoders/sae_ensemble.py:53-77 and its autograd):
//   * one 512-thread workgroup per CU walks a contiguous run of 128 x 128 output tiles
//     (XCD-aware: each XCD gets a contiguous range, i.e. one model's tiles, so W[g] and x stay
//     in that XCD's L2);
//   * waves 0-3 are MFMA waves (2 x 2 of 64 x 64, v_mfma_f32_16x16x32_bf16): they issue the
//     LDS-DMA ring (buffer_load ... lds, NST stages of 64-deep K-tiles, a counted vmcnt keeps
//     NST-2 K-tiles in flight across each barrier, and the ring runs across tile boundaries, so
//     no per-tile prologue is exposed) and keep two accumulator sets: while tile t accumulates,
//     the finished tile t-1 is handed out, two fragments per K-step, through a 2 x 8 KiB LDS
//     staging ring;
//   * waves 4-7 are epilogue waves (one per SIMD, beside an MFMA wave): they read the staged
//     fragments one step later and run the fused epilogue (bias, activation, statistics,
//     activity ballots, 16-byte stores), so the VALU / store work of tile t-1 executes on the
//     SIMDs' vector pipes while the matrix pipes run tile t;
//   * both wave groups execute exactly one s_barrier per step (same trip count, computed from
//     the kernel arguments), so the MFMA waves' vmcnt counts only their own LDS-DMA and the
//     epilogue waves' loads / stores never drain a prefetch.
// Partial-sum layouts are those of the tile kernel (sae_gemm.hip), so the loss / bias / Adam
// kernels consume either.  K must be a multiple of 64 and at least 512 (8 K-steps per tile,
// one staged chunk per step); the tile kernel covers shorter K.
#include "gemm_tiles.h"

namespace scamd {
namespace pg {

constexpr int BM = 128, BN = 128, BK = 64, NT = 512, WI = 4, WJ = 4, NCH = 8;
constexpr int TA = BM * BK * 2, TB = BN * BK * 2, STG = TA + TB;
constexpr int NMW = 4;  // MFMA waves (issue all of the LDS-DMA)
constexpr int PPWA = TA / 1024 / NMW, PPWB = TB / 1024 / NMW, LPT = PPWA + PPWB;
constexpr int SLOT = NMW * 2 * 64 * 16;  // one staged chunk: 4 waves x 2 fragments x 64 lanes x 16 B
// epilogue scratch: column partials [2 regions][2 wave rows][BN] and scalar partials [4][4] (floats)
constexpr int SCR_COL = 2 * 2 * BN;
constexpr int SCR_BYTES = (SCR_COL + 4 * 4) * 4;
template <int NST>
constexpr int lds_bytes() { return NST * STG + 2 * SLOT + SCR_BYTES; }
static_assert(PPWA * NMW * 1024 == TA && PPWB * NMW * 1024 == TB, "tile must split into whole pieces");

__device__ __forceinline__ uint2 pack_bf16(const f32x4_t& v) {
  uint2 r;
  r.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  r.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  return r;
}

// Fragments j and j+1 (32 adjacent columns) of one 16-row block as bf16: after swapping the
// odd 16-lane rows of `a` with the even rows of `b`, lane row q holds 8 contiguous columns --
// {0-7, 16-23, 8-15, 24-31}[q] of the pair -- and stores them with one 16-byte write.
__device__ __forceinline__ void store_pair_bf16(uint16_t* base, uint2 a, uint2 b, int lane) {
  const auto x = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
  const auto y = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
  const int q = lane >> 4;
  const int off = ((q & 1) << 4) | ((q >> 1) << 3);
  *reinterpret_cast<u32x4_t*>(base + off) = u32x4_t{x[0], y[0], x[1], y[1]};
}

// The fragment's 32-byte activity record (four wave ballots): lane l writes dword l & 7;
// the 8 copies of each dword carry identical data, so no lane predicate is needed.
__device__ __forceinline__ void store_ballots(uint64_t* dst, uint64_t b0, uint64_t b1, uint64_t b2, uint64_t b3,
                                              int lane) {
  const int k = lane & 7, h = k >> 1;
  const uint64_t w = h == 0 ? b0 : (h == 1 ? b1 : (h == 2 ? b2 : b3));
  reinterpret_cast<uint32_t*>(dst)[k] = (k & 1) ? (uint32_t)(w >> 32) : (uint32_t)w;
}

struct TileId {
  int pi, g, tm, tn;
};

struct Sched {  // the block's tile range and step count (identical in every wave)
  int t0, ntl, nk, total, per_g, per_p, tiles_n;
  __device__ __forceinline__ TileId tile(int tl) const {
    TileId r;
    const int t = t0 + tl;
    r.pi = t / per_p;
    int rem = t - r.pi * per_p;
    r.g = rem / per_g;
    rem -= r.g * per_g;
    r.tm = rem / tiles_n;
    r.tn = rem - r.tm * tiles_n;
    return r;
  }
  // the chunk the MFMA waves stage at step s: tile tl-1's chunk kt during tile tl's first
  // NCH K-steps, then the last tile's chunks in NCH drain-only steps after the K-loop
  __device__ __forceinline__ bool staged(int s, int& tl, int& c) const {
    if (s < 0) return false;
    if (s < total) {
      const int t = s / nk, kt = s - t * nk;
      tl = t - 1;
      c = kt;
      return t >= 1 && kt < NCH;
    }
    tl = ntl - 1;
    c = s - total;
    return c < NCH;
  }
  // steps: the K-loop, NCH drain-only steps, one to process the last chunk, one to flush
  __device__ __forceinline__ int steps() const { return total + NCH + 2; }
};

// SEG2: the plain F32 / BF16 epilogues with a second K segment (K-concatenated products)
template <bool AK, bool BKM, int EPI, int ACT, int NST, bool SEG2>
__global__ __launch_bounds__(NT, 2) void gemm_p_kernel(GemmParams p) {
  constexpr bool ENC = (EPI == EPI_ENC || EPI == EPI_ENC_CNT || EPI == EPI_ENC_ACT);
  constexpr bool DCK = (EPI == EPI_DC_MASK || EPI == EPI_DC_ACT);
  constexpr bool CHUNK_AUX = (EPI == EPI_DEC) || (EPI == EPI_DC_ACT && ACT == 1);
  __shared__ __attribute__((aligned(16))) char smem[lds_bytes<NST>()];
  char* const stg_base = smem + NST * STG;
  float* const red_c = reinterpret_cast<float*>(stg_base + 2 * SLOT);  // [2][2][BN]
  float* const red_s = red_c + SCR_COL;                                // [4][4]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cw = wid & 3;  // position in the 2 x 2 wave grid (both groups)
  const int wr = cw >> 1, wc = cw & 1;
  Sched sc;
  {
    const int tiles_m = p.M / BM;
    sc.tiles_n = p.N / BN;
    sc.per_g = tiles_m * sc.tiles_n;
    sc.per_p = p.G * sc.per_g;
    const int T = p.nprob * sc.per_p;
    const int nb = gridDim.x;
    const int b = xcd_remap(blockIdx.x, nb);
    sc.t0 = (int)(((long)b * T) / nb);
    sc.ntl = (int)(((long)(b + 1) * T) / nb) - sc.t0;
    sc.nk = p.K1 / BK + (SEG2 ? p.K2 / BK : 0);
    sc.total = sc.ntl * sc.nk;
  }
  if (sc.ntl <= 0) return;
  const int nsteps = sc.steps();

  if (wid < NMW) {
    // =========================================================== MFMA waves
    const int nk = sc.nk, nk1 = p.K1 / BK, total = sc.total;
    uint32_t va0[PPWA], vb0[PPWB], va1[SEG2 ? PPWA : 1], vb1[SEG2 ? PPWB : 1];
    piece_offsets<AK, BK, PPWA>(va0, p.prob[0].a[0].ld, 0, cw, lane);
    piece_offsets<BKM, BK, PPWB>(vb0, p.prob[0].b[0].ld, 0, cw, lane);
    if constexpr (SEG2) {
      piece_offsets<AK, BK, PPWA>(va1, p.prob[0].a[1].ld, 0, cw, lane);
      piece_offsets<BKM, BK, PPWB>(vb1, p.prob[0].b[1].ld, 0, cw, lane);
    }
    // soffset advance per K-step: K-major operands step BK elements, M/N-major BK rows
    const uint32_t sa0 = AK ? BK * 2 : (uint32_t)(BK * p.prob[0].a[0].ld * 2);
    const uint32_t sb0 = BKM ? BK * 2 : (uint32_t)(BK * p.prob[0].b[0].ld * 2);
    const uint32_t sa1 = AK ? BK * 2 : (uint32_t)(BK * p.prob[0].a[1].ld * 2);
    const uint32_t sb1 = BKM ? BK * 2 : (uint32_t)(BK * p.prob[0].b[1].ld * 2);
    int cu_tile = 0, cu_kt = 0, cu_stage = 0;
    i32x4_t ra0, rb0, ra1, rb1;
    uint32_t oa0 = 0, ob0 = 0, oa1 = 0, ob1 = 0;
    auto cursor_tile = [&](int tl) __attribute__((always_inline)) {
      const TileId t = sc.tile(tl);
      const bool p1 = t.pi != 0;
      const Operand A0 = p1 ? p.prob[1].a[0] : p.prob[0].a[0];
      const Operand B0 = p1 ? p.prob[1].b[0] : p.prob[0].b[0];
      const int m0 = t.tm * BM, n0 = t.tn * BN;
      ra0 = make_rsrc(A0.ptr + (long)t.g * A0.sg);
      rb0 = make_rsrc(B0.ptr + (long)t.g * B0.sg);
      oa0 = AK ? (uint32_t)((long)m0 * A0.ld * 2) : (uint32_t)(m0 * 2);
      ob0 = BKM ? (uint32_t)((long)n0 * B0.ld * 2) : (uint32_t)(n0 * 2);
      if constexpr (SEG2) {
        const Operand A1 = p1 ? p.prob[1].a[1] : p.prob[0].a[1];
        const Operand B1 = p1 ? p.prob[1].b[1] : p.prob[0].b[1];
        ra1 = make_rsrc(A1.ptr + (long)t.g * A1.sg);
        rb1 = make_rsrc(B1.ptr + (long)t.g * B1.sg);
        oa1 = AK ? (uint32_t)((long)m0 * A1.ld * 2) : (uint32_t)(m0 * 2);
        ob1 = BKM ? (uint32_t)((long)n0 * B1.ld * 2) : (uint32_t)(n0 * 2);
      }
    };
    auto issue_next = [&]() __attribute__((always_inline)) {
      char* dst = smem + cu_stage * STG;
      if (!SEG2 || cu_kt < nk1) {
        issue_pieces<PPWA>(ra0, va0, oa0 + (uint32_t)cu_kt * sa0, dst, cw);
        issue_pieces<PPWB>(rb0, vb0, ob0 + (uint32_t)cu_kt * sb0, dst + TA, cw);
      } else if constexpr (SEG2) {
        issue_pieces<PPWA>(ra1, va1, oa1 + (uint32_t)(cu_kt - nk1) * sa1, dst, cw);
        issue_pieces<PPWB>(rb1, vb1, ob1 + (uint32_t)(cu_kt - nk1) * sb1, dst + TA, cw);
      }
      cu_stage = cu_stage == NST - 1 ? 0 : cu_stage + 1;
      if (++cu_kt == nk) {
        cu_kt = 0;
        if (++cu_tile < sc.ntl) cursor_tile(cu_tile);
      }
    };

    f32x4_t acc[WI][WJ], accp[WI][WJ];
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
      for (int j = 0; j < WJ; ++j) acc[i][j] = accp[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    auto mfma_step = [&](int stage) __attribute__((always_inline)) {
      const char* la = smem + stage * STG;
      const char* lb = la + TA;
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        bf16x8_t fa[WI], fb[WJ];
#pragma unroll
        for (int j = 0; j < WJ; ++j) fb[j] = load_frag<BKM, BK>(lb, wc * 64 + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < WI; ++i) fa[i] = load_frag<AK, BK>(la, wr * 64 + i * 16, ks, lane);
        // B-side rows as the MFMA's A operand: lane l then holds 4 consecutive OUTPUT columns
        // of one row (acc[i][j][r] = C[16 i + (l & 15)][16 j + 4 (l >> 4) + r] of the wave tile)
#pragma unroll
        for (int i = 0; i < WI; ++i)
#pragma unroll
          for (int j = 0; j < WJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
    };
    // hand chunk C of the finished tile (fragments (C/2, 2(C%2)) and (C/2, 2(C%2)+1)) to the
    // epilogue waves: lane-linear 16-byte records, slot = step & 1
    auto stage_chunk = [&](int c, int slot) __attribute__((always_inline)) {
      f32x4_t* dst = reinterpret_cast<f32x4_t*>(stg_base + slot * SLOT) + cw * 128 + lane;
#define SC_STAGE(C)                                    \
  case C:                                              \
    dst[0] = accp[(C) >> 1][((C) & 1) * 2];            \
    dst[64] = accp[(C) >> 1][((C) & 1) * 2 + 1];       \
    break;
      switch (c) {
        SC_STAGE(0) SC_STAGE(1) SC_STAGE(2) SC_STAGE(3) SC_STAGE(4) SC_STAGE(5) SC_STAGE(6) SC_STAGE(7)
        default: break;
      }
#undef SC_STAGE
    };

    cursor_tile(0);
#pragma unroll
    for (int t = 0; t < NST - 1; ++t)
      if (t < total) issue_next();
    int kt = 0, tl = 0, stage = 0;
    for (int s = 0; s < nsteps; ++s) {
      if (s < total) {
        // K-tile s must have landed; K-tiles s+1 .. s+NST-2 may stay in flight
        const int younger = min(NST - 2, total - 1 - s);
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
      }
      // lgkmcnt(0): this wave's ring reads and staging writes are done; raw barrier (no vmcnt)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (s < total) {
        if (s + NST - 1 < total) issue_next();
        if (tl >= 1 && kt < NCH) stage_chunk(kt, s & 1);
        mfma_step(stage);
        stage = stage == NST - 1 ? 0 : stage + 1;
        if (++kt == nk) {
          kt = 0;
          ++tl;
#pragma unroll
          for (int i = 0; i < WI; ++i)
#pragma unroll
            for (int j = 0; j < WJ; ++j) {
              accp[i][j] = acc[i][j];
              acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            }
        }
      } else if (s - total < NCH) {
        stage_chunk(s - total, s & 1);
      }
    }
    return;
  }

  // ============================================================= epilogue waves
  const int etid = tid - NMW * 64;
  TileId ft{0, 0, 0, 0};  // tile whose block partials wait in LDS for the flush
  bool flush_pend = false;
  float st0 = 0.f, st1 = 0.f;
  f32x4_t cs[WJ], ds[WJ];
  f32x4_t eb[WJ], es2[WJ];  // per-tile columns (bias / gain, threshold s^2) of the current tile
  uint2 xa[2];              // per-chunk auxiliary values (x for the residual, codes for reverse)
#pragma unroll
  for (int j = 0; j < WJ; ++j) {
    cs[j] = ds[j] = eb[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    es2[j] = f32x4_t{1.f, 1.f, 1.f, 1.f};
  }
  xa[0] = xa[1] = make_uint2(0u, 0u);
  const int tiles_m = p.M / BM;

  // auxiliaries of chunk (t, c), loaded one step before it is processed
  auto aux_load = [&](const TileId& t, int c) __attribute__((always_inline)) {
    const int colq = t.tn * BN + wc * 64 + 4 * (lane >> 4);
    if constexpr (ENC) {
      if (c == 0) {
        const long gb = (long)t.g * p.sbias;
#pragma unroll
        for (int j = 0; j < WJ; ++j) {
          eb[j] = *reinterpret_cast<const f32x4_t*>(p.bias + gb + colq + 16 * j);
          if constexpr (ACT == 2) es2[j] = *reinterpret_cast<const f32x4_t*>(p.ascale + gb + colq + 16 * j);
        }
      }
    }
    if constexpr (CHUNK_AUX) {
      const int i = c >> 1, j0 = (c & 1) * 2;
      const long row = t.tm * BM + wr * 64 + i * 16 + (lane & 15);
      const uint16_t* X = p.aux + (long)t.g * p.saux + row * p.ldaux + colq;
      xa[0] = *reinterpret_cast<const uint2*>(X + 16 * j0);
      xa[1] = *reinterpret_cast<const uint2*>(X + 16 * (j0 + 1));
    }
  };

  // The fused epilogue of one staged chunk: fragments (i, J0) and (i, J0 + 1) of wave cw's tile.
  auto process = [&](auto j0c, const f32x4_t (&v)[2], const TileId& t, int i) __attribute__((always_inline)) {
    constexpr int J0 = decltype(j0c)::value;
    const int m0 = t.tm * BM, n0 = t.tn * BN;
    const int row0 = m0 + wr * 64 + i * 16;
    const long row = row0 + (lane & 15);
    const int cbase = n0 + wc * 64;
    const int colq = cbase + 4 * (lane >> 4);
    void* cptr = t.pi ? p.prob[1].c : p.prob[0].c;
    const float alpha = t.pi ? p.prob[1].alpha : p.prob[0].alpha;
    if constexpr (EPI == EPI_F32) {
      float* Cp = reinterpret_cast<float*>(cptr) + (long)t.g * p.sc + row * p.ldc + colq;
      *reinterpret_cast<f32x4_t*>(Cp + 16 * J0) = v[0] * alpha;
      *reinterpret_cast<f32x4_t*>(Cp + 16 * (J0 + 1)) = v[1] * alpha;
    } else if constexpr (EPI == EPI_BF16) {
      uint16_t* Cp = reinterpret_cast<uint16_t*>(cptr) + (long)t.g * p.sc + row * p.ldc;
      store_pair_bf16(Cp + cbase + 16 * J0, pack_bf16(v[0] * alpha), pack_bf16(v[1] * alpha), lane);
    } else if constexpr (ENC) {
      uint16_t* Cp = reinterpret_cast<uint16_t*>(cptr) + (long)t.g * p.sc + row * p.ldc;
      const int nact = p.nactive ? p.nactive[t.g] : p.N;  // masked SAEs: live columns [0, nact)
      uint2 pk[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const int j = J0 + f;
        const int col = colq + 16 * j;
        f32x4_t o;
        bool on[4], ramp[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pre = v[f][r] + eb[j][r];
          float val;
          bool a;
          ramp[r] = false;
          if constexpr (ACT == 1) {
            val = pre > 0.f ? v[f][r] : 0.f;  // relu(pre) - b on the active codes
            a = pre > 0.f;
          } else if constexpr (ACT == 2) {
            const float s2 = es2[j][r];
            const float u = pre / fmaxf(s2, 1e-8f);
            val = (fminf(fmaxf(10.f * (u - 0.9f), 0.f), 1.f) + fmaxf(u - 1.f, 0.f)) * s2;
            a = val > 0.f;
            ramp[r] = u < 1.f;  // slope-10 region, decided on the fp32 pre-activation
          } else {
            val = fmaxf(pre, 0.f);
            a = val > 0.f;
          }
          const bool live = col + r < nact;
          o[r] = live ? val : 0.f;
          on[r] = live && a;
          ramp[r] = ramp[r] && on[r];
          st0 += ACT == 1 ? fabsf(o[r]) : o[r];
          st1 += on[r] ? 1.f : 0.f;
          cs[j][r] += on[r] ? 1.f : 0.f;
        }
        pk[f] = pack_bf16(o);
        const long frag = ((long)t.g * (p.M >> 4) + (row0 >> 4)) * (p.N >> 4) + ((cbase + 16 * j) >> 4);
        store_ballots(p.cmask + frag * 4, __ballot(on[0]), __ballot(on[1]), __ballot(on[2]), __ballot(on[3]), lane);
        if constexpr (ACT == 2)
          store_ballots(p.cmask2 + frag * 4, __ballot(ramp[0]), __ballot(ramp[1]), __ballot(ramp[2]),
                        __ballot(ramp[3]), lane);
      }
      store_pair_bf16(Cp + cbase + 16 * J0, pk[0], pk[1], lane);
    } else if constexpr (EPI == EPI_DEC) {
      uint16_t* Cp = reinterpret_cast<uint16_t*>(cptr) + (long)t.g * p.sc + row * p.ldc;
      uint2 pk[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const uint2 xv = xa[f];
        f32x4_t rv;
        rv[0] = v[f][0] - bf2f(xv.x & 0xFFFF);
        rv[1] = v[f][1] - bf2f(xv.x >> 16);
        rv[2] = v[f][2] - bf2f(xv.y & 0xFFFF);
        rv[3] = v[f][3] - bf2f(xv.y >> 16);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          st0 += rv[r] * rv[r];
          cs[J0 + f][r] += rv[r];  // fp32 column sums (stored only when p.rcol is set)
        }
        pk[f] = pack_bf16(rv);
      }
      store_pair_bf16(Cp + cbase + 16 * J0, pk[0], pk[1], lane);
    } else if constexpr (DCK) {
      uint16_t* Cp = reinterpret_cast<uint16_t*>(cptr) + (long)t.g * p.sc + row * p.ldc;
      const float add = p.l1[t.g] * p.l1_add_scale;
      uint2 pk[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const int j = J0 + f;
        const long frag = ((long)t.g * (p.M >> 4) + (row0 >> 4)) * (p.N >> 4) + ((cbase + 16 * j) >> 4);
        const uint64_t* mk = p.cmask + frag * 4;  // wave-uniform address: scalar loads
        f32x4_t dv;
        if constexpr (EPI == EPI_DC_MASK || ACT == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool on = (mk[r] >> lane) & 1ull;
            dv[r] = on ? v[f][r] + add : 0.f;
            cs[j][r] += dv[r];
          }
        } else if constexpr (ACT == 1) {
          // reverse SAE: sign of the (possibly negative) code for the L1 term, no bias gradient
          const uint2 cv = xa[f];
          const float cvals[4] = {bf2f(cv.x & 0xFFFF), bf2f(cv.x >> 16), bf2f(cv.y & 0xFFFF), bf2f(cv.y >> 16)};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool on = (mk[r] >> lane) & 1ull;
            const float c = cvals[r];
            const float sgn = c > 0.f ? 1.f : (c < 0.f ? -1.f : 0.f);
            dv[r] = on ? v[f][r] + add * sgn : 0.f;
          }
        } else {
          // smooth threshold: slope 10 on the ramp (bit from the encoder's fp32 decision), 1 above;
          // region 1 collects sum_b dL/dc (thr - u thr') = -9 dL/dc on the ramp (scale gradient)
          const uint64_t* rk = p.cmask2 + frag * 4;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool on = (mk[r] >> lane) & 1ull;
            const bool rp = (rk[r] >> lane) & 1ull;
            const float dc = v[f][r] + add;
            dv[r] = on ? dc * (rp ? 10.f : 1.f) : 0.f;
            cs[j][r] += dv[r];
            ds[j][r] += (on && rp) ? -9.f * dc : 0.f;
          }
        }
        pk[f] = pack_bf16(dv);
      }
      store_pair_bf16(Cp + cbase + 16 * J0, pk[0], pk[1], lane);
    }
  };

  // After a tile's last chunk: wave totals -> LDS scratch (read after the next barrier).
  auto finalize = [&](const TileId& t) __attribute__((always_inline)) {
    if constexpr (ENC || EPI == EPI_DEC) {
      const float a0 = wave_sum(st0);
      const float a1 = ENC ? wave_sum(st1) : 0.f;
      if (lane == 0) {
        red_s[cw * 4 + 0] = a0;
        red_s[cw * 4 + 1] = a1;
      }
    }
    bool colstats = DCK;
    if constexpr (EPI == EPI_ENC_CNT) colstats = true;
    if constexpr (EPI == EPI_ENC_ACT) colstats = p.colpart != nullptr;
    if constexpr (EPI == EPI_DEC) colstats = p.rcol != nullptr;
    if constexpr (EPI == EPI_DC_ACT && ACT == 1) colstats = false;
    if (colstats) {
#pragma unroll
      for (int j = 0; j < WJ; ++j) {
        f32x4_t a = cs[j], w = ds[j];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          a[r] = row16_scan(a[r]);
          if constexpr (EPI == EPI_DC_ACT && ACT == 2) w[r] = row16_scan(w[r]);
        }
        if ((lane & 15) == 15) {
          const int c = wc * 64 + j * 16 + 4 * (lane >> 4);
          *reinterpret_cast<f32x4_t*>(red_c + wr * BN + c) = a;
          if constexpr (EPI == EPI_DC_ACT && ACT == 2) *reinterpret_cast<f32x4_t*>(red_c + (2 + wr) * BN + c) = w;
        }
      }
    }
    ft = t;
    flush_pend = true;
  };
  // After a barrier: block totals -> the global partial buffers (one per 128 x 128 tile).
  auto flush = [&]() __attribute__((always_inline)) {
    flush_pend = false;
    const long tile_lin = ((long)ft.g * tiles_m + ft.tm) * sc.tiles_n + ft.tn;
    const long colrow = ((long)ft.g * tiles_m + ft.tm) * p.N + ft.tn * BN;
    if constexpr (ENC) {
      if (etid == 0) {
        p.part[tile_lin * 2 + 0] = red_s[0] + red_s[4] + red_s[8] + red_s[12];
        p.part[tile_lin * 2 + 1] = red_s[1] + red_s[5] + red_s[9] + red_s[13];
      }
      bool counting = EPI == EPI_ENC_CNT;
      if constexpr (EPI == EPI_ENC_ACT) counting = p.colpart != nullptr;
      if (counting && etid < BN) p.colpart[colrow + etid] = red_c[etid] + red_c[BN + etid];
    } else if constexpr (EPI == EPI_DEC) {
      if (etid == 0) p.part[tile_lin] = red_s[0] + red_s[4] + red_s[8] + red_s[12];
      if (p.rcol && etid < BN) p.rcol[colrow + etid] = red_c[etid] + red_c[BN + etid];
    } else if constexpr (DCK) {
      if (etid < BN) {
        if constexpr (EPI == EPI_DC_ACT && ACT == 1) {
          p.colpart[colrow + etid] = 0.f;  // reverse SAEs: the bias gets no gradient through the codes
        } else {
          p.colpart[colrow + etid] = red_c[etid] + red_c[BN + etid];
          if constexpr (EPI == EPI_DC_ACT && ACT == 2)
            if (p.dotpart) p.dotpart[colrow + etid] = red_c[2 * BN + etid] + red_c[3 * BN + etid];
        }
      }
    }
  };

  {
    int tl, c;
    if (sc.staged(0, tl, c)) aux_load(sc.tile(tl), c);
  }
  for (int s = 0; s < nsteps; ++s) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (flush_pend) flush();
    int tl, c;
    if (sc.staged(s - 1, tl, c)) {
      const TileId t = sc.tile(tl);
      const f32x4_t* src = reinterpret_cast<const f32x4_t*>(stg_base + ((s - 1) & 1) * SLOT) + cw * 128 + lane;
      f32x4_t v[2];
      v[0] = src[0];
      v[1] = src[64];
      if (c == 0) {
        st0 = st1 = 0.f;
#pragma unroll
        for (int j = 0; j < WJ; ++j) cs[j] = ds[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
      if (c & 1) process(std::integral_constant<int, 2>{}, v, t, c >> 1);
      else process(std::integral_constant<int, 0>{}, v, t, c >> 1);
      if (c == NCH - 1) finalize(t);
    }
    int tn_, cn;
    if (sc.staged(s, tn_, cn)) aux_load(sc.tile(tn_), cn);  // processed at the next step
  }
}

}  // namespace pg
}  // namespace scamd

using namespace scamd;

namespace {

int g_num_cu = 0;

int num_cu() {
  if (g_num_cu == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    g_num_cu = n;
  }
  return g_num_cu;
}

template <bool AK, bool BKM, int EPI, int ACT, bool SEG2 = false>
int launch_p(const GemmParams& p, int blocks, int nst, hipStream_t stream) {
  if (nst == 4)
    hipLaunchKernelGGL((pg::gemm_p_kernel<AK, BKM, EPI, ACT, 4, SEG2>), dim3(blocks), dim3(pg::NT), 0, stream, p);
  else
    hipLaunchKernelGGL((pg::gemm_p_kernel<AK, BKM, EPI, ACT, 3, SEG2>), dim3(blocks), dim3(pg::NT), 0, stream, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // namespace

extern "C" {

struct ScOperandP {
  const void* ptr;
  long ld, sg;
};

// Arguments of the persistent GEMM (one struct instead of a 40-argument C call).
struct ScGemmArgs {
  int epi, layout, nprob, M, N, K1, K2, G;
  ScOperandP a[4], b[4];  // [nprob][2 K segments]
  void* c[2];
  float alpha[2];
  long ldc, sc;
  const float* bias;
  long sbias;
  const int* nactive;
  const void* aux;
  long ldaux, saux;
  float* part;
  float* colpart;
  const float* l1;
  float l1_add_scale;
  float* dotpart;
  void* cmask;
  void* cmask2;
  float* rcol;
  int act;
  const float* ascale;
  int nst;         // LDS ring stages: 3 (default) or 4
  int max_blocks;  // 0: one workgroup per CU (tests: force several tiles per workgroup)
};

// layout: bit0 = A is K-major, bit1 = B is K-major.  Returns 0 on success.
int sc_gemm_p(const ScGemmArgs* a, hipStream_t stream) {
  const int M = a->M, N = a->N, K1 = a->K1, K2 = a->K2, G = a->G, nprob = a->nprob;
  if (M % pg::BM || N % pg::BN || K1 % pg::BK || K2 % pg::BK || G < 1 || nprob < 1 || nprob > 2) return 1;
  if (K1 + K2 < pg::NCH * pg::BK) return 1;  // at least one staged chunk per K-step
  const bool ak = a->layout & 1, bk = a->layout & 2;
  const int epi = a->epi, act = a->act;
  const bool plain = epi == EPI_F32 || epi == EPI_BF16;
  if (!plain && (K2 != 0 || nprob != 1)) return 1;
  const bool seg2 = K2 > 0;
  // the per-lane DMA offsets are computed once per workgroup: every problem must share the
  // leading dimensions of its K segments
  if (nprob == 2)
    for (int s = 0; s < 2; ++s)
      if (a->a[2 + s].ld != a->a[s].ld || a->b[2 + s].ld != a->b[s].ld) return 9;
  GemmParams p;
  for (int i = 0; i < nprob; ++i) {
    for (int s = 0; s < 2; ++s) {
      p.prob[i].a[s] = {reinterpret_cast<const uint16_t*>(a->a[i * 2 + s].ptr), a->a[i * 2 + s].ld, a->a[i * 2 + s].sg};
      p.prob[i].b[s] = {reinterpret_cast<const uint16_t*>(a->b[i * 2 + s].ptr), a->b[i * 2 + s].ld, a->b[i * 2 + s].sg};
    }
    p.prob[i].c = a->c[i];
    p.prob[i].alpha = a->alpha[i];
  }
  if (nprob == 1) p.prob[1] = p.prob[0];
  p.nprob = nprob;
  p.M = M; p.N = N; p.K1 = K1; p.K2 = K2; p.G = G;
  p.ldc = a->ldc; p.sc = a->sc;
  p.bias = a->bias; p.sbias = a->sbias; p.nactive = a->nactive;
  p.aux = reinterpret_cast<const uint16_t*>(a->aux); p.ldaux = a->ldaux; p.saux = a->saux;
  p.part = a->part; p.colpart = a->colpart; p.l1 = a->l1; p.l1_add_scale = a->l1_add_scale;
  p.dotpart = a->dotpart; p.dc_tied = 0;
  p.cmask = reinterpret_cast<uint64_t*>(a->cmask);
  p.cmask2 = reinterpret_cast<uint64_t*>(a->cmask2);
  p.rcol = a->rcol;
  for (int i = 0; i < 2; ++i) p.adam[i] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  p.lr = nullptr; p.step = nullptr; p.b1 = p.b2 = p.eps = 0.f; p.dot_tm = 0; p.dot_scale = 0.f;
  p.ksplit = 1; p.split_stride = 0;
  p.act = act; p.ascale = a->ascale;
  // argument checks for the fused epilogues (a bad pointer faults the node, not the call)
  const bool enc = epi == EPI_ENC || epi == EPI_ENC_CNT || epi == EPI_ENC_ACT;
  if (enc && (!ak || !bk || !a->bias || !a->part || !a->cmask)) return 4;
  if (epi == EPI_ENC_CNT && !a->colpart) return 4;
  if ((epi == EPI_ENC_ACT || epi == EPI_DC_ACT) && (act < 1 || act > 2)) return 4;
  if (act == 2 && (epi == EPI_ENC_ACT || epi == EPI_DC_ACT) && !a->cmask2) return 4;
  if (act == 2 && epi == EPI_ENC_ACT && !a->ascale) return 4;
  if (epi == EPI_DEC && (!ak || bk || !a->aux || !a->part)) return 4;
  if ((epi == EPI_DC_MASK || epi == EPI_DC_ACT) && (!ak || !bk || !a->cmask || !a->colpart || !a->l1)) return 4;
  if (epi == EPI_DC_ACT && act == 1 && !a->aux) return 4;
  const long tiles = (long)nprob * G * (M / pg::BM) * (N / pg::BN);
  long blocks = num_cu();
  if (a->max_blocks > 0 && blocks > a->max_blocks) blocks = a->max_blocks;
  if (blocks > tiles) blocks = tiles;
  const int nst = a->nst == 4 ? 4 : 3;
#define SC_P(AKV, BKV, E, A) return launch_p<AKV, BKV, E, A>(p, (int)blocks, nst, stream)
  if (seg2) {  // K-concatenated weight gradients of tied dictionaries (M/N-major operands)
    if (epi != EPI_F32 || ak || bk) return 5;
    return launch_p<false, false, EPI_F32, 0, true>(p, (int)blocks, nst, stream);
  }
  switch (epi) {
    case EPI_F32:
      if (ak && bk) SC_P(true, true, EPI_F32, 0);
      if (ak) SC_P(true, false, EPI_F32, 0);
      if (bk) SC_P(false, true, EPI_F32, 0);
      SC_P(false, false, EPI_F32, 0);
    case EPI_BF16:
      if (ak && bk) SC_P(true, true, EPI_BF16, 0);
      if (ak) SC_P(true, false, EPI_BF16, 0);
      if (bk) SC_P(false, true, EPI_BF16, 0);
      SC_P(false, false, EPI_BF16, 0);
    case EPI_ENC: SC_P(true, true, EPI_ENC, 0);
    case EPI_ENC_CNT: SC_P(true, true, EPI_ENC_CNT, 0);
    case EPI_ENC_ACT:
      if (act == 1) SC_P(true, true, EPI_ENC_ACT, 1);
      SC_P(true, true, EPI_ENC_ACT, 2);
    case EPI_DEC: SC_P(true, false, EPI_DEC, 0);
    case EPI_DC_MASK: SC_P(true, true, EPI_DC_MASK, 0);
    case EPI_DC_ACT:
      if (act == 1) SC_P(true, true, EPI_DC_ACT, 1);
      SC_P(true, true, EPI_DC_ACT, 2);
    default: return 2;
  }
#undef SC_P
}

}  // extern "C"
