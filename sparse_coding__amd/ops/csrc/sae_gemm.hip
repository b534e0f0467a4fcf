// Grouped bf16 MFMA GEMM with fused sparse-autoencoder epilogues (gfx950).
//
// One launch covers every model of an ensemble (the "group" axis G) and, for
// the weight-gradient pass, two independent problems at once.  This replaces
// the reference's torch.vmap(torch.func.grad(loss)) over stacked parameters
// (reference autoencoders/ensemble.py:119-123) with explicit kernels:
//
//   EPI_ENC : c = relu(x W_e^T + b)  (+ masked tail), bf16 store, L1/L0 partials
//             (autoencoders/sae_ensemble.py:54-56, :354 masked_fill_)
//   EPI_DEC : R = c W_hat - x, bf16 store, sum(R^2) partials
//             (autoencoders/sae_ensemble.py:58-62)
//   EPI_DC  : dpre_s = 1[c>0] * (R W_hat^T + lambda*d/2), bf16 store, column-sum
//             partials for the bias gradient (autograd of :54-64, Appendix A of SURVEY)
//   EPI_F32 : C = alpha * acc (fp32), used for dW = c^T R and dW_e = dpre^T x
//   EPI_BF16: C = alpha * acc (bf16), generic inference GEMM
//
// Tiling: 128x128 block tile, 256 threads = 4 waves in a 2x2 grid, each wave
// owns a 64x64 sub-tile = 4x4 v_mfma_f32_16x16x32_bf16 accumulators.  Operands
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
#include "common.h"

namespace scamd {

constexpr int BM = 128, BN = 128, NT = 256;

enum { EPI_ENC = 0, EPI_DEC = 1, EPI_DC = 2, EPI_F32 = 3, EPI_BF16 = 4 };

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
  __builtin_amdgcn_s_waitcnt((N & 15) | (((N >> 4) & 3) << 14) | 0x70 | 0xF00);
}

// Per-lane byte offsets (relative to the operand's group base) of the 1 KiB
// LDS-DMA pieces this wave fills for K-tile 0; later tiles add a scalar soffset.
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
      voff[i] = (uint32_t)(((long)(r0 + row) * ld + ch * 8) * 2);
    } else {
      const int row = piece * 4 + (lane >> 4);
      const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
      voff[i] = (uint32_t)(((long)row * ld + r0 + ch * 8) * 2);
    }
  }
}

template <int PPW>
__device__ __forceinline__ void issue_pieces(__amdgpu_buffer_rsrc_t rs, const uint32_t* voff, uint32_t soff,
                                             char* lds_tile, int wid) {
#pragma unroll
  for (int i = 0; i < PPW; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds_tile + (wid * PPW + i) * 1024),
                                            16, voff[i], soff, 0, 0);
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

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const uint16_t* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7FFFFFFF, 0x00020000);
}

template <bool AK, bool BKM, int EPI, int BKT, int NST>
__global__ __launch_bounds__(NT) void sae_gemm_kernel(GemmParams p) {
  constexpr int TB = 128 * BKT * 2;  // bytes per operand tile
  constexpr int PPW = TB / 1024 / 4; // LDS-DMA pieces per wave per operand tile
  constexpr int LPT = 2 * PPW;       // DMA instructions per wave per K-tile
  __shared__ __attribute__((aligned(16))) char smem[NST * 2 * TB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int tiles_m = p.M / BM, tiles_n = p.N / BN;
  const int per_prob = tiles_m * tiles_n * p.G;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int pi = bid / per_prob;
  int rem = bid - pi * per_prob;
  const int g = rem / (tiles_m * tiles_n);
  rem -= g * tiles_m * tiles_n;
  const int tm = rem / tiles_n, tn = rem - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // Resolve the problem's operands with selects (a dynamically indexed kernarg
  // struct would be copied to scratch).
  const bool p1 = pi != 0;
  const Operand oa0 = p1 ? p.prob[1].a[0] : p.prob[0].a[0];
  const Operand oa1 = p1 ? p.prob[1].a[1] : p.prob[0].a[1];
  const Operand ob0 = p1 ? p.prob[1].b[0] : p.prob[0].b[0];
  const Operand ob1 = p1 ? p.prob[1].b[1] : p.prob[0].b[1];
  void* cptr = p1 ? p.prob[1].c : p.prob[0].c;
  const float alpha = p1 ? p.prob[1].alpha : p.prob[0].alpha;

  const int nk1 = p.K1 / BKT, nk = nk1 + p.K2 / BKT;
  // per-lane DMA source offsets for both K segments (segment 2 only for K-concat GEMMs)
  uint32_t va0[PPW], vb0[PPW], va1[PPW], vb1[PPW];
  piece_offsets<AK, BKT, PPW>(va0, oa0.ld, m0, wid, lane);
  piece_offsets<BKM, BKT, PPW>(vb0, ob0.ld, n0, wid, lane);
  piece_offsets<AK, BKT, PPW>(va1, oa1.ld, m0, wid, lane);
  piece_offsets<BKM, BKT, PPW>(vb1, ob1.ld, n0, wid, lane);
  const __amdgpu_buffer_rsrc_t ra0 = make_rsrc(oa0.ptr + (long)g * oa0.sg);
  const __amdgpu_buffer_rsrc_t rb0 = make_rsrc(ob0.ptr + (long)g * ob0.sg);
  const __amdgpu_buffer_rsrc_t ra1 = make_rsrc(oa1.ptr + (long)g * oa1.sg);
  const __amdgpu_buffer_rsrc_t rb1 = make_rsrc(ob1.ptr + (long)g * ob1.sg);
  // soffset advance per K-tile: K-major operands step BKT elements, M/N-major BKT rows
  const uint32_t sa0 = AK ? BKT * 2 : (uint32_t)(BKT * oa0.ld * 2), sa1 = AK ? BKT * 2 : (uint32_t)(BKT * oa1.ld * 2);
  const uint32_t sb0 = BKM ? BKT * 2 : (uint32_t)(BKT * ob0.ld * 2), sb1 = BKM ? BKT * 2 : (uint32_t)(BKT * ob1.ld * 2);

#define SC_ISSUE(t)                                                           \
  do {                                                                        \
    char* dst_ = smem + ((t) % NST) * 2 * TB;                                 \
    if ((t) < nk1) {                                                          \
      issue_pieces<PPW>(ra0, va0, (uint32_t)(t) * sa0, dst_, wid);            \
      issue_pieces<PPW>(rb0, vb0, (uint32_t)(t) * sb0, dst_ + TB, wid);       \
    } else {                                                                  \
      issue_pieces<PPW>(ra1, va1, (uint32_t)((t) - nk1) * sa1, dst_, wid);    \
      issue_pieces<PPW>(rb1, vb1, (uint32_t)((t) - nk1) * sb1, dst_ + TB, wid); \
    }                                                                         \
  } while (0)

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (t < nk) SC_ISSUE(t);

  for (int kt = 0; kt < nk; ++kt) {
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
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of the stage being recycled are done
    __builtin_amdgcn_s_barrier();        // raw barrier: no implicit vmcnt(0), DMAs stay in flight
    if (kt + NST - 1 < nk) SC_ISSUE(kt + NST - 1);
    const char* la = smem + (kt % NST) * 2 * TB;
    const char* lb = la + TB;
#pragma unroll
    for (int ks = 0; ks < BKT / 32; ++ks) {
      bf16x8_t fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = load_frag<AK, BKT>(la, wr * 64 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = load_frag<BKM, BKT>(lb, wc * 64 + j * 16, ks, lane);
      // Operands swapped (B-side rows as the MFMA's A): each lane then holds
      // 4 consecutive OUTPUT COLUMNS of one output row, so the epilogue
      // issues 8/16-byte vector stores instead of 2-byte scatters.
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
#undef SC_ISSUE
  __syncthreads();  // all reads of the ring done before smem is reused below

  // ------------------------------------------------------------------ epilogue
  // acc[i][j][r] = C[row][col0 + r] with row = m0 + wr*64 + i*16 + (lane&15),
  // col0 = n0 + wc*64 + j*16 + 4*(lane>>4).
  const int rowb = m0 + wr * 64 + (lane & 15);
  const int colb = n0 + wc * 64 + 4 * (lane >> 4);
  float* red = reinterpret_cast<float*>(smem);  // free after the barrier above

  if constexpr (EPI == EPI_F32) {
    float* C = reinterpret_cast<float*>(cptr) + (long)g * p.sc;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4_t v = acc[i][j] * alpha;
        *reinterpret_cast<f32x4_t*>(C + (long)(rowb + i * 16) * p.ldc + colb + j * 16) = v;
      }
    return;
  }
  if constexpr (EPI == EPI_BF16) {
    uint16_t* C = reinterpret_cast<uint16_t*>(cptr) + (long)g * p.sc;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        ushort4 h;
        h.x = f2bf(alpha * acc[i][j][0]); h.y = f2bf(alpha * acc[i][j][1]);
        h.z = f2bf(alpha * acc[i][j][2]); h.w = f2bf(alpha * acc[i][j][3]);
        *reinterpret_cast<ushort4*>(C + (long)(rowb + i * 16) * p.ldc + colb + j * 16) = h;
      }
    return;
  }
  // Column partial sums (ENC: on-counts, DC: bias gradient): reduce each lane's
  // 4x4 values over rows, then across the 16 lanes sharing a column group, then
  // across the two wave rows through LDS.  Deterministic; one store per column.
  auto column_partials = [&](f32x4_t (&cs)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = cs[j][r];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        cs[j][r] = v;
      }
    __syncthreads();
    if ((lane & 15) == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<f32x4_t*>(red + wr * 128 + wc * 64 + j * 16 + 4 * (lane >> 4)) = cs[j];
    }
    __syncthreads();
    if (tid < 128) p.colpart[((long)g * tiles_m + tm) * p.N + n0 + tid] = red[tid] + red[128 + tid];
  };

  if constexpr (EPI == EPI_ENC) {
    uint16_t* C = reinterpret_cast<uint16_t*>(cptr) + (long)g * p.sc;
    const float* bias = p.bias + (long)g * p.sbias;
    const int nact = p.nactive ? p.nactive[g] : p.N;
    const bool masked = nact < p.N;  // block-uniform: only masked ensembles pay for the test
    float l1 = 0.f, l0 = 0.f;
    f32x4_t cnt[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = colb + j * 16;
      const f32x4_t bj = *reinterpret_cast<const f32x4_t*>(bias + col);
      cnt[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f32x4_t v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(acc[i][j][r] + bj[r], 0.f);
        if (masked) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (col + r < nact) ? v[r] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          l1 += v[r];
          const float on = v[r] > 0.f ? 1.f : 0.f;
          l0 += on;
          cnt[j][r] += on;
        }
        *reinterpret_cast<ushort4*>(C + (long)(rowb + i * 16) * p.ldc + col) =
            make_ushort4(f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3]));
      }
    }
    if (p.colpart) column_partials(cnt);
    l1 = block_sum_256(l1, red + 512);
    l0 = block_sum_256(l0, red + 512);
    if (tid == 0) {
      float* part = p.part + ((long)g * tiles_m * tiles_n + tm * tiles_n + tn) * 2;
      part[0] = l1;
      part[1] = l0;
    }
    return;
  }
  if constexpr (EPI == EPI_DEC) {
    uint16_t* C = reinterpret_cast<uint16_t*>(cptr) + (long)g * p.sc;
    const uint16_t* X = p.aux + (long)g * p.saux;
    float se = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long row = rowb + i * 16;
        const int col = colb + j * 16;
        const ushort4 xv = *reinterpret_cast<const ushort4*>(X + row * p.ldaux + col);
        const float r0 = acc[i][j][0] - bf2f(xv.x), r1 = acc[i][j][1] - bf2f(xv.y);
        const float r2 = acc[i][j][2] - bf2f(xv.z), r3 = acc[i][j][3] - bf2f(xv.w);
        *reinterpret_cast<ushort4*>(C + row * p.ldc + col) = make_ushort4(f2bf(r0), f2bf(r1), f2bf(r2), f2bf(r3));
        se += r0 * r0 + r1 * r1 + r2 * r2 + r3 * r3;
      }
    se = block_sum_256(se, red);
    if (tid == 0) p.part[(long)g * tiles_m * tiles_n + tm * tiles_n + tn] = se;
    return;
  }
  if constexpr (EPI == EPI_DC) {
    uint16_t* C = reinterpret_cast<uint16_t*>(cptr) + (long)g * p.sc;
    const uint16_t* Cin = p.aux + (long)g * p.saux;
    const float add = p.l1[g] * p.l1_add_scale;
    f32x4_t cs[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cs[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long row = rowb + i * 16;
        const int col = colb + j * 16;
        const ushort4 cv = *reinterpret_cast<const ushort4*>(Cin + row * p.ldaux + col);
        const uint16_t cvs[4] = {cv.x, cv.y, cv.z, cv.w};
        f32x4_t dv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dv[r] = cvs[r] != 0 ? acc[i][j][r] + add : 0.f;  // c is a ReLU output: nonzero <=> > 0
          cs[j][r] += dv[r];
        }
        *reinterpret_cast<ushort4*>(C + row * p.ldc + col) =
            make_ushort4(f2bf(dv[0]), f2bf(dv[1]), f2bf(dv[2]), f2bf(dv[3]));
      }
    }
    column_partials(cs);
    return;
  }
}

}  // namespace scamd

using namespace scamd;

// ------------------------------------------------------------------ C ABI
extern "C" {

struct ScOperand {
  const void* ptr;
  long ld, sg;
};

// layout: bit0 = A is K-major, bit1 = B is K-major.
int sc_gemm(int epi, int layout, int nprob, int M, int N, int K1, int K2, int G,
            const ScOperand* a /* [nprob][2] */, const ScOperand* b /* [nprob][2] */,
            void* const* c /* [nprob] */, const float* alpha /* [nprob] */, long ldc, long sc,
            const float* bias, long sbias, const int* nactive, const void* aux, long ldaux,
            long saux, float* part, float* colpart, const float* l1, float l1_add_scale,
            int cfg, hipStream_t stream) {
  if (M % BM || N % BN || K1 % 64 || K2 % 64 || nprob < 1 || nprob > 2 || G < 1) return 1;
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
  const int grid = (M / BM) * (N / BN) * G * nprob;
  const bool ak = layout & 1, bk = layout & 2;

#define SC_LAUNCH(AKV, BKV, E)                                                                    \
  switch (cfg) {                                                                                  \
    case 1: hipLaunchKernelGGL((sae_gemm_kernel<AKV, BKV, E, 32, 3>), dim3(grid), dim3(NT), 0, stream, p); break; \
    case 2: hipLaunchKernelGGL((sae_gemm_kernel<AKV, BKV, E, 32, 4>), dim3(grid), dim3(NT), 0, stream, p); break; \
    default: hipLaunchKernelGGL((sae_gemm_kernel<AKV, BKV, E, 64, 2>), dim3(grid), dim3(NT), 0, stream, p); break; \
  }
#define SC_EPI(AKV, BKV)                                   \
  switch (epi) {                                           \
    case EPI_ENC: SC_LAUNCH(AKV, BKV, EPI_ENC); break;     \
    case EPI_DEC: SC_LAUNCH(AKV, BKV, EPI_DEC); break;     \
    case EPI_DC: SC_LAUNCH(AKV, BKV, EPI_DC); break;       \
    case EPI_F32: SC_LAUNCH(AKV, BKV, EPI_F32); break;     \
    case EPI_BF16: SC_LAUNCH(AKV, BKV, EPI_BF16); break;   \
    default: return 2;                                     \
  }
  if (ak && bk) { SC_EPI(true, true) }
  else if (ak && !bk) { SC_EPI(true, false) }
  else if (!ak && !bk) { SC_EPI(false, false) }
  else { SC_EPI(false, true) }
#undef SC_EPI
#undef SC_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
