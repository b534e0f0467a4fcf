// Fused code gradient + encoder weight gradient of the untied ReLU SAE step (gfx950).
//
// The step's kernels 3 and 4b were
//   dc     dpre[g] = 1[c > 0] (R[g] W_hat[g]^T + l1[g] d / 2)      [B, n] bf16 -> HBM (67 MB at
//                                                                   the headline shape)
//   wgrad  g_enc[g] = alpha dpre[g]^T x                             (reads dpre back)
// (reference math: the autograd of autoencoders/sae_ensemble.py:53-77).  Here ONE launch never
// materialises dpre: a workgroup owns 64 features j of one model and streams the batch in
// 32-row chunks, flash-attention-backward style --
//   S[32, 64]  = R_chunk W_hat[j]^T          K = d, split over the 4 waves (each its d/4 slice;
//                                             W_hat[j] slice held in VGPRs for the whole launch)
//   P          = 1[mask] (S + l1 d / 2)       the 4 K-partials summed through LDS, the activity
//                                             bits from the encoder's bitmask, bf16 into LDS
//   g_enc[j]  += P^T x_chunk                  K = 32 rows, each wave its d/4 output columns
// and the bias-gradient column sums of P per 128-row slot (the layout the step tail reads).
// Per workgroup the batch is read once (R and x, 4 MB at B = 2048, d = 512 -- L2-resident per
// XCD: the XCD-aware order gives each XCD one model's 32 feature blocks), 64 FLOP per byte.
//
// Operands reach LDS by LDS-DMA (buffer_load ... lds, issued from asm so the compiler does not
// drain them) into per-wave private slabs -- each wave reads only the R columns of its own K
// slice and the x columns of its own output slice -- so their hand-off needs no barrier, only
// the wave's own counted vmcnt; two barriers per chunk remain (partial-S exchange, P).
//
//   per wave, chunk c:  wait R(c) | GEMM1 (32 MFMA) | issue R(c+1), x(c+1) | S partials -> LDS |
//                       barrier | sum 4 partials, mask, P -> LDS | barrier | wait x(c) |
//                       GEMM2 (32 MFMA)
//
// LDS: R slabs 4 x 8 KB, x slabs 4 x 2 x 8 KB, S exchange 32 KB, P image 8 KB, the activity
// words of a 2048-row batch segment 16 KB, 1 KB junk for the L2 warm-up touches = 153 KB.
#include "gemm_tiles.h"

namespace scamd {

struct DcwArgs {
  const uint16_t* R;       // [G][B][D] residual (bf16)
  const uint16_t* W;       // [G][n][D] normalised decoder shadow (bf16)
  const uint16_t* X;       // [B][D] batch (bf16), or per model with stride sx
  long sx;
  const uint64_t* cmask;   // [G][B/64][n/64][64] encoder activity words (sae_gemm_kernel.h mask_bit)
  const float* l1;         // [G]
  float add_scale;         // l1[g] * add_scale is added to active entries (= d / 2)
  float alpha;             // g_enc scale (2 grad_scale / (B d))
  float* genc;             // [G][n][D] fp32 out
  float* colpart;          // [G][B/128][n] fp32 out: column sums of P per 128-row slot
  int G, B, n;
};

constexpr int DCW_JN = 64, DCW_BT = 32, DCW_SEG = 2048;
constexpr int DCW_PF = 4;  // chunks ahead of the L2 warm-up touches

// L2 warm-up: one dword per lane from 64 distinct 128-byte lines, LDS-DMA'd into a junk LDS
// word (no VGPR is written, so nothing has to stay reserved while it is in flight).  Counted
// by vmcnt like every other transfer (the explicit waits below include it).
__device__ __forceinline__ void touch_lines(const i32x4_t& rs, uint32_t voff, uint32_t soff, char* junk) {
  asm volatile(
      "s_mov_b32 m0, %0\n\t"
      "s_nop 0\n\t"
      "buffer_load_dword %1, %2, %3 offen lds"
      :
      : "s"((uint32_t)reinterpret_cast<uintptr_t>(junk)), "v"(voff), "s"(rs), "s"(soff)
      : "memory", "m0");
}

template <int D>
__global__ __launch_bounds__(256, 1) void sae_dcw_kernel(DcwArgs a) {
  constexpr int KW = D / 4;            // GEMM1 K slice per wave
  constexpr int KS = KW / 32;          // its k-steps
  constexpr int CT = (D / 4) / 16;     // GEMM2 16-column output tiles per wave
  constexpr int SLAB = DCW_BT * KW * 2;  // per-wave R / x slab bytes (8 KB at D = 512)
  constexpr int PPW = SLAB / 1024;       // DMA pieces per slab
  static_assert(KW == 128, "per-wave slabs are 128 columns wide (one M/N-major half image)");
  constexpr int R_OFF = 0;                          // [4 waves][SLAB]
  constexpr int X_OFF = R_OFF + 4 * SLAB;           // [2 bufs][4 waves][SLAB]
  constexpr int S_OFF = X_OFF + 8 * SLAB;           // [4 w][4 t][2 i][64] f32x4
  constexpr int P_OFF = S_OFF + 4 * 4 * 2 * 64 * 16;  // [32 b][256 B] image (64 j used)
  constexpr int M_OFF = P_OFF + DCW_BT * 256;       // [32 blocks][64] u64
  constexpr int J_OFF = M_OFF + (DCW_SEG / 64) * 512;  // [4 waves][256 B] junk (L2 touches)
  __shared__ __attribute__((aligned(16))) char smem[J_OFF + 4 * 256];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nj = a.n / DCW_JN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int g = bid / nj, j0 = (bid - g * nj) * DCW_JN;
  const int B = a.B, n = a.n, nc = B / DCW_BT, tm = B / 128;
  const float add = a.l1[g] * a.add_scale;

  // ---- this wave's W_hat slice [64 j][KW k] as MFMA fragments (lane: row 16t + (l&15), k 8(l>>4))
  bf16x8_t fw[4][KS];
  {
    const uint16_t* Wg = a.W + ((long)g * n + j0 + (lane & 15)) * D + w * KW + 8 * (lane >> 4);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int s = 0; s < KS; ++s) fw[t][s] = *reinterpret_cast<const bf16x8_t*>(Wg + (long)t * 16 * D + 32 * s);
  }
  __syncthreads();  // (a real vmcnt(0): the compiler's wait tracking then sees fw complete in the loop)

  // ---- DMA source offsets (bytes, relative to the chunk's first row; soffset advances rows)
  // R slab: [32 rows][16 chunks of 16 B] with chunk ^= row & 15 (ds_read_b128 16-lane groups
  // of 16 rows x one chunk hit 16 distinct 16-byte bank groups)
  uint32_t vr[PPW];
#pragma unroll
  for (int p = 0; p < PPW; ++p) {
    const int row = 4 * p + (lane >> 4), ch = (lane & 15) ^ (row & 15);
    vr[p] = (uint32_t)(row * D + w * KW + 8 * ch) * 2u;
  }
  // x slab: the M/N-major [32 k-rows][128 columns] half image of gemm_tiles.h (mmaj_off)
  uint32_t vx[PPW];
  piece_offsets<false, 32, PPW>(vx, D, 0, w, lane);
  const i32x4_t rsR = make_rsrc(a.R + (long)g * B * D);
  const i32x4_t rsX = make_rsrc(a.X + (long)g * a.sx);
  char* const rslab = smem + R_OFF;
  char* const xs0 = smem + X_OFF;
  f32x4_t* const sred = reinterpret_cast<f32x4_t*>(smem + S_OFF);
  char* const pimg = smem + P_OFF;
  const uint64_t* const mimg = reinterpret_cast<const uint64_t*>(smem + M_OFF);

  f32x4_t acc[4][CT];
#pragma unroll
  for (int it = 0; it < 4; ++it)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[it][ct] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float cs[4] = {0.f, 0.f, 0.f, 0.f};

  // L2 warm-up of chunk c + DCW_PF: the XCD's 32 workgroups stream the same R[g] and x rows in near
  // lockstep, so without it every chunk starts with the full MALL / HBM latency; waves 0-1 touch
  // the R chunk, 2-3 the x chunk (256 lines each), lanes spread over the lines by feature block
  const int tq = (((j0 / DCW_JN) * 2 + (w & 1)) * 64 + lane) & 255;
  const uint32_t vt = (uint32_t)((tq >> 3) * D * 2 + (tq & 7) * 128);
  char* const junk = smem + J_OFF + w * 256;
  auto touch = [&](int c) {
    const int cc = min(c, nc - 1);  // always issued: the vmcnt bookkeeping counts it
    touch_lines(w < 2 ? rsR : rsX, vt, (uint32_t)(cc * DCW_BT * D * 2), junk);
  };

  auto issue_r = [&](int c) { issue_pieces<PPW>(rsR, vr, (uint32_t)(c * DCW_BT * D * 2), rslab, w); };
  auto issue_x = [&](int c) {
    issue_pieces<PPW>(rsX, vx, (uint32_t)(c * DCW_BT * D * 2), xs0 + (c & 1) * 4 * SLAB, w);
  };

  for (int c = 0; c < nc; ++c) {
    if ((c & (DCW_SEG / DCW_BT - 1)) == 0) {
      // activity words of the next 2048-row segment -> LDS (a full drain, once per segment)
      __syncthreads();
      const int nb = min(DCW_SEG, B - c * DCW_BT) / 64;
      const uint64_t* src = a.cmask + ((long)g * (B / 64) + c / 2) * (n / 64) * 64 + (j0 / 64) * 64;
      uint64_t* dst = reinterpret_cast<uint64_t*>(smem + M_OFF);
      uint64_t mv[DCW_SEG / 256];  // all loads in flight, then the LDS stores
#pragma unroll
      for (int q = 0; q < DCW_SEG / 256; ++q) {
        const int e = min(threadIdx.x + 256 * q, nb * 64 - 1);  // (clamped: no branch per load)
        mv[q] = src[(long)(e >> 6) * (n / 64) * 64 + (e & 63)];
      }
#pragma unroll
      for (int q = 0; q < DCW_SEG / 256; ++q) dst[threadIdx.x + 256 * q] = mv[q];
      if (c == 0) {
        issue_r(0);
        issue_x(0);
        for (int t = 1; t <= DCW_PF; ++t) touch(t);
      }
      __syncthreads();  // (drains this wave's DMAs as well)
    }
    // ---- R(c) landed (younger: x(c) and one L2 touch, issued after it)
    wait_vmcnt<PPW + 1>();
    // ---- GEMM1: S partial over this wave's K slice; lane gets S[b = 16 i + (l&15)][j = 16 t + 4(l>>4) + r]
    f32x4_t sacc[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) sacc[t][0] = sacc[t][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const char* rs = rslab + w * SLAB;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      bf16x8_t fr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = 16 * i + (lane & 15), ch = (4 * s + (lane >> 4)) ^ (row & 15);
        fr[i] = *reinterpret_cast<const bf16x8_t*>(rs + row * 256 + ch * 16);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 2; ++i) sacc[t][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[t][s], fr[i], sacc[t][i], 0, 0, 0);
    }
    // ---- prefetch: the next chunk's R slab (its reads above are complete) and x slab (the other
    // buffer: last read by this wave's GEMM2 two chunks ago)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (c + 1 < nc) {
      issue_r(c + 1);
      issue_x(c + 1);
      touch(c + 1 + DCW_PF);
    }
    // ---- exchange the K partials: wave w sums the 16-column tile t = w of all four
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 2; ++i) sred[((w * 4 + t) * 2 + i) * 64 + lane] = sacc[t][i];
    lds_barrier();
    const uint64_t mw = mimg[((c & (DCW_SEG / DCW_BT - 1)) >> 1) * 64 + lane];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f32x4_t sv = sred[((0 * 4 + w) * 2 + i) * 64 + lane];
#pragma unroll
      for (int ww = 1; ww < 4; ++ww) sv += sred[((ww * 4 + w) * 2 + i) * 64 + lane];
      const int ii = 2 * (c & 1) + i;
      ushort4 h;
      float pv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool on = (mw >> (((ii * 4 + w) * 4) + r)) & 1ull;
        pv[r] = on ? sv[r] + add : 0.f;
        cs[r] += pv[r];
      }
      h.x = f2bf(pv[0]); h.y = f2bf(pv[1]); h.z = f2bf(pv[2]); h.w = f2bf(pv[3]);
      // P[b][j .. j+3] into the M/N-major image (k = b rows, columns j)
      const int b = 16 * i + (lane & 15), j = 16 * w + 4 * (lane >> 4);
      *reinterpret_cast<ushort4*>(pimg + mmaj_off(b, j >> 3) + (j & 7) * 2) = h;
    }
    lds_barrier();
    // ---- x(c) landed (younger: R(c+1), x(c+1), the touch)
    if (c + 1 < nc) wait_vmcnt<2 * PPW + 1>();
    else wait_vmcnt<0>();
    // ---- GEMM2: g_enc[j][col] += P^T x; lane gets [j = 16 it + (l&15)][col = 16 ct + 4(l>>4) + r]
    bf16x8_t fp[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) fp[it] = load_frag<false, 32>(pimg, 16 * it, 0, lane);
    const char* xb = xs0 + (c & 1) * 4 * SLAB;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const bf16x8_t fx = load_frag<false, 32>(xb, w * 128 + 16 * ct, 0, lane);
#pragma unroll
      for (int it = 0; it < 4; ++it) acc[it][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fx, fp[it], acc[it][ct], 0, 0, 0);
    }
    // ---- bias-gradient column sums, one slot per 128 rows
    if ((c & 3) == 3) {
      f32x4_t v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = row16_scan(cs[r]);
        cs[r] = 0.f;
      }
      if ((lane & 15) == 15)
        *reinterpret_cast<f32x4_t*>(a.colpart + ((long)g * tm + (c >> 2)) * n + j0 + 16 * w + 4 * (lane >> 4)) = v;
    }
  }
  // ---- g_enc rows j0 .. j0+63, this wave's columns
  float* out = a.genc + ((long)g * n + j0 + (lane & 15)) * D + w * 128 + 4 * (lane >> 4);
#pragma unroll
  for (int it = 0; it < 4; ++it)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
      *reinterpret_cast<f32x4_t*>(out + (long)it * 16 * D + 16 * ct) = acc[it][ct] * a.alpha;
}

}  // namespace scamd

using namespace scamd;

extern "C" {

// Returns 0 on success, 2 when the shape is not supported (the caller keeps the two-kernel path).
int sc_sae_dcw(const void* R, const void* W, const void* X, long sx, const void* cmask, const float* l1,
               float add_scale, float alpha, float* genc, float* colpart, int G, int B, int n, int d,
               hipStream_t stream) {
  if (d != 512 || n % DCW_JN || B % 128 || G < 1) return 2;
  DcwArgs a;
  a.R = static_cast<const uint16_t*>(R);
  a.W = static_cast<const uint16_t*>(W);
  a.X = static_cast<const uint16_t*>(X);
  a.sx = sx;
  a.cmask = static_cast<const uint64_t*>(cmask);
  a.l1 = l1;
  a.add_scale = add_scale;
  a.alpha = alpha;
  a.genc = genc;
  a.colpart = colpart;
  a.G = G;
  a.B = B;
  a.n = n;
  hipLaunchKernelGGL((sae_dcw_kernel<512>), dim3((unsigned)(G * (n / DCW_JN))), dim3(256), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // extern "C"
