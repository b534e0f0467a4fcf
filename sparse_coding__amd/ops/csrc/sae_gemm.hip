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
// Tiling: 128x128 block tile, BK = 64, 256 threads = 4 waves in a 2x2 grid,
// each wave owns a 64x64 sub-tile = 4x4 v_mfma_f32_16x16x32_bf16 accumulators.
// Operands are staged global -> VGPR -> LDS with a two-buffer pipeline (the
// next K-tile's global loads are issued before the current tile's MFMAs).
// K-major operands are read with ds_read_b128, M/N-major operands with the
// gfx950 transposing read ds_read_b64_tr_b16, so c^T R style products need no
// transposed copies in HBM.  Both LDS images are XOR-swizzled to avoid bank
// conflicts.
#include "common.h"

namespace scamd {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = 128 * 64 * 2;  // 16 KiB per operand tile

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

// LDS image of a K-major tile [128 rows][64 k] bf16: 128-byte rows, 8 chunks
// of 16 bytes, chunk index XORed with (row>>1)&7.
__device__ __forceinline__ int kmaj_off(int row, int ch) {
  return row * 128 + ((ch ^ ((row >> 1) & 7)) << 4);
}
// LDS image of an M/N-major tile [64 k][128 cols] bf16: 256-byte rows, 16
// chunks, swizzle that keeps the transposed 4x16 block reads conflict free.
__device__ __forceinline__ int mmaj_off(int row, int ch) {
  return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}

template <bool KMAJ>
__device__ __forceinline__ void stage_load(const uint16_t* __restrict__ base, long ld, int r0,
                                           int k0, uint4 (&regs)[4], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = tid + NT * i;
    if constexpr (KMAJ) {
      const int row = id >> 3, ch = id & 7;
      regs[i] = *reinterpret_cast<const uint4*>(base + (long)(r0 + row) * ld + k0 + ch * 8);
    } else {
      const int row = id >> 4, ch = id & 15;
      regs[i] = *reinterpret_cast<const uint4*>(base + (long)(k0 + row) * ld + r0 + ch * 8);
    }
  }
}

template <bool KMAJ>
__device__ __forceinline__ void stage_store(char* lds, const uint4 (&regs)[4], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = tid + NT * i;
    int off;
    if constexpr (KMAJ) off = kmaj_off(id >> 3, id & 7);
    else off = mmaj_off(id >> 4, id & 15);
    *reinterpret_cast<uint4*>(lds + off) = regs[i];
  }
}

// Fragment for v_mfma_f32_16x16x32_bf16: lane l holds X[r = rbase + (l&15)][k = 8(l>>4) + j].
template <bool KMAJ>
__device__ __forceinline__ bf16x8_t load_frag(const char* lds, int rbase, int ks, int lane) {
  if constexpr (KMAJ) {
    const int row = rbase + (lane & 15);
    const int ch = ks * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8_t*>(lds + kmaj_off(row, ch));
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

template <bool AK, bool BKM, int EPI>
__global__ __launch_bounds__(NT) void sae_gemm_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2][2][TILE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
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
  const Problem& P = p.prob[pi];

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk1 = p.K1 / BK, nk = nk1 + p.K2 / BK;
  uint4 ra[4], rb[4];

  auto load_tile = [&](int kt) {
    const int seg = kt < nk1 ? 0 : 1;
    const int k0 = (kt - (seg ? nk1 : 0)) * BK;
    const Operand& A = P.a[seg];
    const Operand& B = P.b[seg];
    stage_load<AK>(A.ptr + (long)g * A.sg, A.ld, m0, k0, ra, tid);
    stage_load<BKM>(B.ptr + (long)g * B.sg, B.ld, n0, k0, rb, tid);
  };

  load_tile(0);
  stage_store<AK>(smem[0][0], ra, tid);
  stage_store<BKM>(smem[0][1], rb, tid);
  __syncthreads();

  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) load_tile(kt + 1);
    const char* la = smem[buf][0];
    const char* lb = smem[buf][1];
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8_t fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = load_frag<AK>(la, wr * 64 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = load_frag<BKM>(lb, wc * 64 + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      stage_store<AK>(smem[buf ^ 1][0], ra, tid);
      stage_store<BKM>(smem[buf ^ 1][1], rb, tid);
    }
    __syncthreads();
    buf ^= 1;
  }

  // ------------------------------------------------------------------ epilogue
  // Accumulator element (i, j, r) sits at row m0 + wr*64 + i*16 + (lane>>4)*4 + r,
  // column n0 + wc*64 + j*16 + (lane&15).
  const int rowb = m0 + wr * 64 + (lane >> 4) * 4;
  const int colb = n0 + wc * 64 + (lane & 15);
  float* red = reinterpret_cast<float*>(smem[0][0]);  // free after the last barrier

  if constexpr (EPI == EPI_F32) {
    float* C = reinterpret_cast<float*>(P.c) + (long)g * p.sc;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          C[(long)(rowb + i * 16 + r) * p.ldc + colb + j * 16] = P.alpha * acc[i][j][r];
    return;
  }
  if constexpr (EPI == EPI_BF16) {
    uint16_t* C = reinterpret_cast<uint16_t*>(P.c) + (long)g * p.sc;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          C[(long)(rowb + i * 16 + r) * p.ldc + colb + j * 16] = f2bf(P.alpha * acc[i][j][r]);
    return;
  }
  if constexpr (EPI == EPI_ENC) {
    uint16_t* C = reinterpret_cast<uint16_t*>(P.c) + (long)g * p.sc;
    const float* bias = p.bias + (long)g * p.sbias;
    const int nact = p.nactive ? p.nactive[g] : p.N;
    float l1 = 0.f, l0 = 0.f;
    float cnt[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = colb + j * 16;
      const float bj = bias[col];
      const bool live = col < nact;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = fmaxf(acc[i][j][r] + bj, 0.f);
          v = live ? v : 0.f;
          const uint16_t h = f2bf(v);
          C[(long)(rowb + i * 16 + r) * p.ldc + col] = h;
          const float vb = bf2f(h);  // stats on the stored (bf16) code
          l1 += vb;
          const float on = vb > 0.f ? 1.f : 0.f;
          l0 += on;
          cnt[j] += on;
        }
    }
    l1 = block_sum_256(l1, red + 512);
    l0 = block_sum_256(l0, red + 512);
    const int tile = tm * tiles_n + tn;
    if (tid == 0) {
      float* part = p.part + ((long)g * tiles_m * tiles_n + tile) * 2;
      part[0] = l1;
      part[1] = l0;
    }
    if (p.colpart) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cnt[j] += __shfl_xor(cnt[j], 16, 64);
        cnt[j] += __shfl_xor(cnt[j], 32, 64);
      }
      if (lane < 16) {
#pragma unroll
        for (int j = 0; j < 4; ++j) red[wr * 128 + wc * 64 + j * 16 + lane] = cnt[j];
      }
      __syncthreads();
      if (tid < 128)
        p.colpart[((long)g * tiles_m + tm) * p.N + n0 + tid] = red[tid] + red[128 + tid];
    }
    return;
  }
  if constexpr (EPI == EPI_DEC) {
    uint16_t* C = reinterpret_cast<uint16_t*>(P.c) + (long)g * p.sc;
    const uint16_t* X = p.aux + (long)g * p.saux;
    float se = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long row = rowb + i * 16 + r;
          const int col = colb + j * 16;
          const float res = acc[i][j][r] - bf2f(X[row * p.ldaux + col]);
          C[row * p.ldc + col] = f2bf(res);
          se += res * res;
        }
    se = block_sum_256(se, red);
    if (tid == 0) p.part[(long)g * tiles_m * tiles_n + tm * tiles_n + tn] = se;
    return;
  }
  if constexpr (EPI == EPI_DC) {
    uint16_t* C = reinterpret_cast<uint16_t*>(P.c) + (long)g * p.sc;
    const uint16_t* Cin = p.aux + (long)g * p.saux;
    const float add = p.l1[g] * p.l1_add_scale;
    float cs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long row = rowb + i * 16 + r;
          const int col = colb + j * 16;
          const float cv = bf2f(Cin[row * p.ldaux + col]);
          const float d = cv > 0.f ? acc[i][j][r] + add : 0.f;
          const uint16_t h = f2bf(d);
          C[row * p.ldc + col] = h;
          cs[j] += bf2f(h);
        }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cs[j] += __shfl_xor(cs[j], 16, 64);
      cs[j] += __shfl_xor(cs[j], 32, 64);
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < 4; ++j) red[wr * 128 + wc * 64 + j * 16 + lane] = cs[j];
    }
    __syncthreads();
    if (tid < 128) p.colpart[((long)g * tiles_m + tm) * p.N + n0 + tid] = red[tid] + red[128 + tid];
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
            hipStream_t stream) {
  if (M % BM || N % BN || K1 % BK || K2 % BK || nprob < 1 || nprob > 2 || G < 1) return 1;
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

#define SC_LAUNCH(AKV, BKV, E) \
  hipLaunchKernelGGL((sae_gemm_kernel<AKV, BKV, E>), dim3(grid), dim3(NT), 0, stream, p)
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
