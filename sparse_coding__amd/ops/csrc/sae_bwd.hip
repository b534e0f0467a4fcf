// Row-block weight gradient + Adam for SAE ensembles (gfx950): the last two stages of the
// training step fused into ONE launch, so the fp32 weight gradients never touch HBM.
//
// Reference math (autoencoders/sae_ensemble.py:53-77 under vmap(grad), then torchopt adam,
// autoencoders/ensemble.py:175-193; Appendix A of SURVEY.md):
//   dW_e   = alpha * dpre^T x                 (encoder, untied)
//   dW_hat = alpha * c^T R                    (decoder, row-normalised inside the loss)
//   dW_d[j] = (dW_hat[j] - w_hat[j] <w_hat[j], dW_hat[j]>) / |W_d[j]|   (norm Jacobian)
//   tied:  dW_hat = alpha * (dpre^T x + c^T R), then the same Jacobian on the shared dictionary
// followed by Adam (fp32 masters and moments) and the bf16 shadows the next step's GEMMs read
// (decoder / tied dictionary: row-normalised, with its row norms).
//
// Decomposition: one workgroup owns F = 64 dictionary rows of one model and ALL d columns, and
// streams the batch through LDS in chunks of 32 rows (double-buffered LDS-DMA: the dpre / c
// column tiles [32 x 64] and the x / R row tiles [32 x d]).  Wave w of NW = d / 64 holds the
// fp32 accumulators of columns [64 w, 64 w + 64) for all 64 rows (16 MFMA 16x16 tiles per
// product, 128 accumulator registers untied); every operand fragment is a transposing LDS read
// (ds_read_b64_tr_b16), so neither dpre^T nor R^T exists in HBM.  Because a workgroup ends
// with complete rows of BOTH gradients in registers, the whole Adam update -- including the
// norm Jacobian's row dot and the new row norm, reduced across the NW waves through LDS --
// runs in the epilogue: compared with wgrad GEMM -> fp32 gradient in HBM -> Adam kernel this
// removes the gradient's write + read (2 x 4 B per parameter) and the partial-sum buffers
// (dotpart / sqpart) of the previous design.
//
// Grid: G * n / 64 workgroups (256 for the headline 8 x 2048 ensemble: one per CU), mapped so
// the n / 64 workgroups of one model share an XCD (its R and x tiles stay in that L2).
#include "common.h"

namespace scamd {

namespace bwd {

constexpr int F = 64;      // dictionary rows per workgroup
constexpr int BC = 32;     // batch rows per chunk (= MFMA K)
constexpr int TROW = F * 2;  // bytes per row of a [BC x F] column tile

// LDS images.  Row tiles [BC][d] bf16 (1 KB rows at d = 512): 16-byte chunk c of row r sits at
// c ^ sw_row(r); column tiles [BC][F] (128-byte rows): chunk c at c ^ sw_col(r).  Both keep the
// transposing reads conflict-free: a 32-lane bank group of ds_read_b64_tr_b16 reads rows
// {0-3, 8-11} (+16, +4) at one 32-byte column segment, and the XOR sends those 8 rows to 8
// distinct 32-byte bank windows (row tiles: 1 KB rows all start at bank 0; column tiles:
// odd rows start at bank 32, so 4 windows per row parity suffice).
__device__ __forceinline__ int sw_row(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }
__device__ __forceinline__ int sw_col(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }

struct Params {
  int G, B, n, d;
  const uint16_t* c;     // [G][B][n] bf16 codes
  const uint16_t* dpre;  // [G][B][n] bf16 code gradient (masked, in units of 2/(B d))
  const uint16_t* R;     // [G][B][d] bf16 residual
  const uint16_t* x;     // [B][d] (sx = 0) or [G][B][d] bf16 encoder input
  long sx;
  float alpha;           // 2 grad_scale / (B d)
  // Adam state.  Untied: set 0 = encoder (plain rows), set 1 = decoder (row-normalised).
  // Tied: set 1 only (the dictionary), set 0 unused.
  float* p[2];
  float* m[2];
  float* v[2];
  uint16_t* shadow[2];
  float* norms;          // [G][n] row norms of the normalised set (written)
  const float* lr;       // [G]
  const int* step;       // completed steps (t = *step + 1)
  float b1, b2, eps;
  const int* nactive;    // optional [G] live rows (masked ensembles; multiples of 64)
};

template <int NW, bool TIED>
struct Cfg {
  static constexpr int D = NW * 64;
  static constexpr int NT = NW * 64;
  static constexpr int ROWT = BC * D * 2;                // bytes of one [BC][D] row tile
  static constexpr int COLT = BC * TROW;                 // bytes of one [BC][F] column tile (4 KB)
  static constexpr int OFF_X = 0, OFF_R = ROWT, OFF_DP = 2 * ROWT, OFF_C = 2 * ROWT + COLT;
  static constexpr int STAGE = 2 * ROWT + 2 * COLT;
  // LDS-DMA pieces (1 KB each) per chunk: 2 row tiles of BC rows x (D / 512) pieces, and the
  // two column tiles (4 pieces each)
  static constexpr int ROW_PIECES = BC * D * 2 / 1024;  // per row tile
  static constexpr int PIECES = 2 * ROW_PIECES + 8;
  static_assert(PIECES % NW == 0, "pieces must split evenly over the waves");
  static constexpr int PPW = PIECES / NW;                // DMA instructions per wave per chunk
};

// LDS-DMA pieces: piece `idx` of a chunk (wave-uniform) targets operand piece_op(idx) at LDS
// byte offset piece_lds(idx) of the stage; its per-lane source offset (bytes, relative to the
// operand's group base, chunk 0) is precomputed once (piece_voff) and later chunks only add a
// scalar soffset.  The destination is lane-linear, so the swizzle is applied to the SOURCE:
// lane L fills physical chunk L and fetches the logical chunk the image places there.
template <class C>
__device__ __forceinline__ int piece_op(int idx) {  // 0 = x, 1 = R, 2 = dpre, 3 = c
  return idx < 2 * C::ROW_PIECES ? idx / C::ROW_PIECES : (idx - 2 * C::ROW_PIECES < 4 ? 2 : 3);
}
template <class C>
__device__ __forceinline__ uint32_t piece_lds(int idx) {
  if (idx < 2 * C::ROW_PIECES) {
    const int op = idx / C::ROW_PIECES;
    return (op == 0 ? C::OFF_X : C::OFF_R) + (idx - op * C::ROW_PIECES) * 1024;
  }
  const int q = idx - 2 * C::ROW_PIECES;
  return (q < 4 ? C::OFF_DP : C::OFF_C) + (q & 3) * 1024;
}
template <class C>
__device__ __forceinline__ uint32_t piece_voff(int idx, int lane, int f0, int n) {
  if (idx < 2 * C::ROW_PIECES) {
    const int q = idx % C::ROW_PIECES;               // piece within the row tile
    const int bytes = q * 1024 + lane * 16;          // lane-linear destination
    const int row = bytes / (C::D * 2);
    const int pch = (bytes - row * C::D * 2) >> 4;   // physical chunk
    const int lch = pch ^ sw_row(row);               // logical chunk it holds
    return (uint32_t)(row * C::D + lch * 8) * 2u;
  }
  const int q = (idx - 2 * C::ROW_PIECES) & 3;       // dpre pieces 0-3, then c pieces 0-3
  const int row = q * 8 + (lane >> 3);
  const int lch = (lane & 7) ^ sw_col(row);
  return (uint32_t)(row * n + f0 + lch * 8) * 2u;
}

typedef int i32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4_t rsrc(const uint16_t* base) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32) & 0xFFFF);
  r[2] = 0x7FFFFFFF;
  r[3] = 0x00020000;
  return r;
}

// one LDS-DMA piece (64 lanes x 16 B -> 1 KB contiguous at LDS byte address `lds`); issued from
// inline asm so hipcc does not insert vmcnt(0) waits before later ds_reads (see gemm_tiles.h)
__device__ __forceinline__ void dma(const i32x4_t& rs, uint32_t voff, uint32_t soff, uint32_t lds) {
  asm volatile(
      "s_mov_b32 m0, %0\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %3 offen lds"
      :
      : "s"(lds), "v"(voff), "s"(rs), "s"(soff)
      : "memory", "m0");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// MFMA operand fragment by transposing reads from a [BC][*] tile whose 16-byte chunks are
// XOR-swizzled per row: lane l gets T[k = 8 (l >> 4) + 0..7][col = cb + (l & 15)] (k = batch
// row), i.e. the K-major fragment of T^T.  `rowb` = bytes per tile row.
template <bool ROWT>
__device__ __forceinline__ bf16x8_t tr_frag(const char* tile, int rowb, int cb, int lane) {
  const int li = lane & 15, q = li >> 2, p = li & 3, g = lane >> 4;
  const int ch = (cb >> 3) + (p >> 1);
  const int within = (p & 1) * 8;
  const int r0 = 8 * g + q, r1 = r0 + 4;
  const int s0 = ROWT ? sw_row(r0) : sw_col(r0), s1 = ROWT ? sw_row(r1) : sw_col(r1);
  i16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(SC_LDS(i16x4_t, tile + r0 * rowb + ((ch ^ s0) << 4) + within));
  i16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(SC_LDS(i16x4_t, tile + r1 * rowb + ((ch ^ s1) << 4) + within));
  typedef short i16x8_t __attribute__((ext_vector_type(8)));
  i16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float at(const float4& v, int r) { return r == 0 ? v.x : r == 1 ? v.y : r == 2 ? v.z : v.w; }
__device__ __forceinline__ void set(float4& v, int r, float x) {
  if (r == 0) v.x = x; else if (r == 1) v.y = x; else if (r == 2) v.z = x; else v.w = x;
}

}  // namespace bwd

template <int NW, bool TIED>
__global__ __launch_bounds__(NW * 64) void sae_bwd_adam_kernel(bwd::Params P) {
  using namespace bwd;
  using C = Cfg<NW, TIED>;
  constexpr int D = C::D;
  __shared__ __attribute__((aligned(16))) char smem[2 * C::STAGE];  // 2 stages; reductions reuse stage 0

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nfb = P.n / F;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int g = lin / nfb, fb = lin - g * nfb, f0 = fb * F;
  if (P.nactive && f0 >= P.nactive[g]) return;  // dead rows of a masked model: no gradient, no update

  // ---- DMA setup: PPW pieces per wave, fixed per-lane offsets, per-operand soffset per chunk
  const uint16_t* xg = P.x + (long)g * P.sx;
  const i32x4_t rs_x = rsrc(xg), rs_r = rsrc(P.R + (long)g * P.B * D);
  const i32x4_t rs_dp = rsrc(P.dpre + (long)g * P.B * P.n), rs_c = rsrc(P.c + (long)g * P.B * P.n);
  uint32_t voff[C::PPW];
#pragma unroll
  for (int i = 0; i < C::PPW; ++i) voff[i] = piece_voff<C>(w * C::PPW + i, lane, f0, P.n);
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>(smem);
  const uint32_t step_row = BC * D * 2, step_col = BC * P.n * 2;  // soffset per chunk
  auto issue = [&](int k) {
    const uint32_t st = lds0 + (k & 1) * C::STAGE;
#pragma unroll
    for (int i = 0; i < C::PPW; ++i) {
      const int idx = w * C::PPW + i;  // wave-uniform: operand, LDS slot and soffset are scalar
      const int op = piece_op<C>(idx);
      const i32x4_t rs = op == 0 ? rs_x : op == 1 ? rs_r : op == 2 ? rs_dp : rs_c;
      const uint32_t so = (op < 2 ? step_row : step_col) * (uint32_t)k;
      dma(rs, voff[i], so, st + piece_lds<C>(idx));
    }
  };

  constexpr int NA = TIED ? 1 : 2;  // accumulator sets: [0] = x-side (dW_e / tied), [1] = R-side
  f32x4_t acc[NA][4][4];
#pragma unroll
  for (int s = 0; s < NA; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[s][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nch = P.B / BC;
  issue(0);
  for (int k = 0; k < nch; ++k) {
    wait_vm<0>();                                         // chunk k landed (this wave's pieces)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // ... everyone's; stage k^1 free
    if (k + 1 < nch) issue(k + 1);
    const char* st = smem + (k & 1) * C::STAGE;
    bf16x8_t xf[4], rf[4], df[4], cf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      xf[j] = tr_frag<true>(st + C::OFF_X, D * 2, 64 * w + 16 * j, lane);
      rf[j] = tr_frag<true>(st + C::OFF_R, D * 2, 64 * w + 16 * j, lane);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      df[i] = tr_frag<false>(st + C::OFF_DP, TROW, 16 * i, lane);
      cf[i] = tr_frag<false>(st + C::OFF_C, TROW, 16 * i, lane);
    }
    // acc[i][j][r] = sum_b T1[b][f = 16 i + (l & 15)] T2[b][col = 64 w + 16 j + 4 (l >> 4) + r]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[0][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[j], df[i], acc[0][i][j], 0, 0, 0);
        acc[NA - 1][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rf[j], cf[i], acc[NA - 1][i][j], 0, 0, 0);
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // LDS free for the reductions

  // ---------------------------------------------------------------- Adam epilogue
  // lane l holds rows f0 + 16 i + (l & 15), columns 64 w + 16 j + 4 (l >> 4) + 0..3
  const float t = (float)(*P.step + 1);
  const float bc1 = 1.f - __powf(P.b1, t), bc2 = 1.f - __powf(P.b2, t);
  const float lr = P.lr[g], stp = lr / bc1, rbc2 = 1.f / bc2;
  const float b1 = P.b1, b2 = P.b2, omb1 = 1.f - P.b1, omb2 = 1.f - P.b2, eps = P.eps;
  const float alpha = P.alpha;
  const int rl = lane & 15, cq = 4 * (lane >> 4);
  auto off = [&](int i, int j) { return ((long)g * P.n + f0 + 16 * i + rl) * D + 64 * w + 16 * j + cq; };

  if constexpr (!TIED) {  // encoder: plain rows
    float* p = P.p[0];
    float* m = P.m[0];
    float* v = P.v[0];
    uint16_t* sh = P.shadow[0];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float4 pv[4], mv[4], vv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long o = off(i, j);
        pv[j] = ld4(p + o);
        mv[j] = ld4(m + o);
        vv[j] = ld4(v + o);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long o = off(i, j);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gk = acc[0][i][j][r] * alpha;
          const float mk = b1 * at(mv[j], r) + omb1 * gk;
          const float vk = b2 * at(vv[j], r) + omb2 * gk * gk;
          set(mv[j], r, mk);
          set(vv[j], r, vk);
          set(pv[j], r, at(pv[j], r) - stp * mk / (sqrtf(vk * rbc2) + eps));
        }
        st4(p + o, pv[j]);
        st4(m + o, mv[j]);
        st4(v + o, vv[j]);
        *reinterpret_cast<ushort4*>(sh + o) =
            make_ushort4(f2bf(pv[j].x), f2bf(pv[j].y), f2bf(pv[j].z), f2bf(pv[j].w));
      }
    }
  }

  // row-normalised set (decoder, or the tied dictionary): norm Jacobian + Adam + shadow
  {
    constexpr int S = NA - 1;
    float* p = P.p[1];
    float* m = P.m[1];
    float* v = P.v[1];
    uint16_t* sh = P.shadow[1];
    float* red = reinterpret_cast<float*>(smem);  // [2][NW][F] partial (dot, |w|^2) per wave and row
    float4 pv[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) pv[i][j] = ld4(p + off(i, j));
    // per-row partial <w, g> and |w|^2 over this wave's 64 columns (the 4 lanes of a row: l ^ 16, 32)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float dot = 0.f, ss = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pw = at(pv[i][j], r);
          dot += pw * acc[S][i][j][r];
          ss += pw * pw;
        }
      dot += __shfl_xor(dot, 16, 64);
      dot += __shfl_xor(dot, 32, 64);
      ss += __shfl_xor(ss, 16, 64);
      ss += __shfl_xor(ss, 32, 64);
      if (lane < 16) {
        red[(0 * NW + w) * F + 16 * i + lane] = dot;
        red[(1 * NW + w) * F + 16 * i + lane] = ss;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float gs[4], ws[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float dot = 0.f, ss = 0.f;
#pragma unroll
      for (int u = 0; u < NW; ++u) {
        dot += red[(0 * NW + u) * F + 16 * i + rl];
        ss += red[(1 * NW + u) * F + 16 * i + rl];
      }
      dot *= alpha;
      const float nrm = sqrtf(ss);
      if (nrm > 1e-8f) {
        const float inv = 1.f / nrm;
        gs[i] = inv;                    // g' = (g - w_hat <w_hat, g>) / |w|
        ws[i] = dot * inv * inv * inv;  //    = g / |w| - w <w, g> / |w|^3
      } else {
        gs[i] = 1e8f;                   // clamp(min=1e-8) has zero derivative below the floor
        ws[i] = 0.f;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // red is reused below
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float4 mv[4], vv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long o = off(i, j);
        mv[j] = ld4(m + o);
        vv[j] = ld4(v + o);
      }
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long o = off(i, j);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pw = at(pv[i][j], r);
          const float gk = acc[S][i][j][r] * alpha * gs[i] - pw * ws[i];
          const float mk = b1 * at(mv[j], r) + omb1 * gk;
          const float vk = b2 * at(vv[j], r) + omb2 * gk * gk;
          set(mv[j], r, mk);
          set(vv[j], r, vk);
          const float pn = pw - stp * mk / (sqrtf(vk * rbc2) + eps);
          set(pv[i][j], r, pn);
          ss += pn * pn;
        }
        st4(p + o, pv[i][j]);
        st4(m + o, mv[j]);
        st4(v + o, vv[j]);
      }
      ss += __shfl_xor(ss, 16, 64);
      ss += __shfl_xor(ss, 32, 64);
      if (lane < 16) red[w * F + 16 * i + lane] = ss;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float ss = 0.f;
#pragma unroll
      for (int u = 0; u < NW; ++u) ss += red[u * F + 16 * i + rl];
      const float nrm = fmaxf(sqrtf(ss), 1e-8f);
      const float sc = 1.f / nrm;
      if (w == 0 && lane < 16) P.norms[(long)g * P.n + f0 + 16 * i + lane] = nrm;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 q = pv[i][j];
        *reinterpret_cast<ushort4*>(sh + off(i, j)) =
            make_ushort4(f2bf(q.x * sc), f2bf(q.y * sc), f2bf(q.z * sc), f2bf(q.w * sc));
      }
    }
  }
}

}  // namespace scamd

using namespace scamd;

extern "C" {

// Fused weight gradient + Adam (see the header comment).  Returns 0 on success; 1 = shape not
// supported (d must be 256 or 512, B % 32, n % 64), 3 = launch error.
int sc_bwd_adam(int tied, int G, int B, int n, int d, const void* c, const void* dpre, const void* R,
                const void* x, long sx, float alpha, float* const* p, float* const* m, float* const* v,
                void* const* shadow, float* norms, const float* lr, const int* step, float b1, float b2,
                float eps, const int* nactive, hipStream_t stream) {
  if (B % bwd::BC || n % bwd::F || G < 1 || (d != 256 && d != 512)) return 1;
  bwd::Params P;
  P.G = G; P.B = B; P.n = n; P.d = d;
  P.c = reinterpret_cast<const uint16_t*>(c);
  P.dpre = reinterpret_cast<const uint16_t*>(dpre);
  P.R = reinterpret_cast<const uint16_t*>(R);
  P.x = reinterpret_cast<const uint16_t*>(x);
  P.sx = sx;
  P.alpha = alpha;
  for (int s = 0; s < 2; ++s) {
    P.p[s] = p[s]; P.m[s] = m[s]; P.v[s] = v[s];
    P.shadow[s] = reinterpret_cast<uint16_t*>(shadow[s]);
  }
  P.norms = norms; P.lr = lr; P.step = step; P.b1 = b1; P.b2 = b2; P.eps = eps; P.nactive = nactive;
  const dim3 grid((unsigned)(G * (n / bwd::F)));
#define SC_BWD(NWV, TV) hipLaunchKernelGGL((sae_bwd_adam_kernel<NWV, TV>), grid, dim3(NWV * 64), 0, stream, P)
  if (d == 512) {
    if (tied) SC_BWD(8, true); else SC_BWD(8, false);
  } else {
    if (tied) SC_BWD(4, true); else SC_BWD(4, false);
  }
#undef SC_BWD
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
