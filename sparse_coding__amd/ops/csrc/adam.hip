// Fused Adam for stacked dictionary parameters (gfx950).
//
// Reference semantics: torchopt 0.7.1 `adam` vmapped over the model axis
// (reference autoencoders/ensemble.py:94-95, :123, :182-191), with the decoder
// row normalisation done *inside* the loss (autoencoders/sae_ensemble.py:58-59),
// so the gradient reaching the raw decoder goes through the norm Jacobian:
//     dW[j] = (dW_hat[j] - W_hat[j] <W_hat[j], dW_hat[j]>) / max(|W[j]|, 1e-8)
// One wave owns one dictionary row (d elements).  In a single HBM pass it
// applies the norm Jacobian, the Adam update, recomputes the row norm and
// writes the bf16 shadow (normalised for NORM rows) that the next step's
// MFMA GEMMs read.  Bias / loss bookkeeping runs in a second tiny kernel that
// also reduces the deterministic per-tile partials written by the GEMM
// epilogues (no float atomics anywhere in the step).
#include "common.h"
#include "row_adam.h"

#include <algorithm>
#include <stdlib.h>

namespace scamd {

struct AdamRows {
  float* p;         // [rows][d] fp32 master
  const void* g;    // [rows][d] gradient (w.r.t. the normalised row if norm): fp32, or bf16 (GBF)
  float* m;
  float* v;
  uint16_t* shadow; // [rows][d] bf16 copy for the GEMMs (normalised if norm)
  float* norms;     // [rows] optional: new row norms
  int rows;
  int norm;         // 1: row-normalised parameter (decoder / tied dict)
};

struct AdamArgs {
  AdamRows set[2];
  int nset;
  int d;
  int rows_per_model;
  long row0;        // global row index of row 0 (row-sharded updates): lr index = (row0 + row) / rows_per_model
  int nsplit;       // the gradient arrives as `nsplit` split-K partial slabs ...
  long gstride;     // ... `gstride` elements apart (summed here; 1 = a plain gradient)
  const float* lr;  // per model
  float b1, b2, eps, bc1, bc2;
  const int* step;  // optional device step counter (graph-capturable); t = *step + 1
  const int* live;  // optional per-model live row count (masked ensembles): rows past it are skipped
};

template <int NV, bool GBF = false>
__device__ __forceinline__ void adam_row(const AdamArgs& a, long wave) {
  const int lane = threadIdx.x & 63;
  long row = wave;
  int s = 0;
  if (row >= a.set[0].rows) {
    row -= a.set[0].rows;
    s = 1;
    if (s >= a.nset || row >= a.set[1].rows) return;
  }
  const AdamRows& R = a.set[s];
  const long grow = row + a.row0;
  if (a.live && (int)(grow % a.rows_per_model) >= a.live[grow / a.rows_per_model]) return;  // dead row: zero grad
  const float lr = a.lr[grow / a.rows_per_model];
  float bc1 = a.bc1, bc2 = a.bc2;
  if (a.step) bias_corrections(a.b1, a.b2, *a.step + 1, bc1, bc2);
  adam_row_core<NV, GBF>(R.p, R.g, R.m, R.v, R.shadow, R.norms, row, R.norm, a.nsplit, a.gstride, lr, a.b1, a.b2,
                         a.eps, bc1, bc2, lane);
}

template <int NV, bool GBF = false>
__global__ __launch_bounds__(256) void adam_rows_kernel(AdamArgs a) {
  adam_row<NV, GBF>(a, (long)blockIdx.x * 4 + (threadIdx.x >> 6));
}

// Writes a bf16 (optionally row-normalised) shadow of fp32 rows; used at init
// and after any out-of-band parameter change (e.g. FISTA basis update).
__global__ __launch_bounds__(256) void shadow_rows_kernel(const float* p, uint16_t* shadow, float* norms,
                                                          long rows, int d, int norm) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* P = p + row * d;
  float ss = 0.f;
  for (int e = lane * 4; e < d; e += 256) {
    const float4 v = *reinterpret_cast<const float4*>(P + e);
    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  float sc = 1.f;
  if (norm) {
    ss = wave_sum(ss);
    const float nrm = fmaxf(sqrtf(ss), 1e-8f);
    sc = 1.f / nrm;
    if (norms && lane == 0) norms[row] = nrm;
  }
  for (int e = lane * 4; e < d; e += 256) {
    const float4 v = *reinterpret_cast<const float4*>(P + e);
    ushort4 h;
    h.x = f2bf(v.x * sc);
    h.y = f2bf(v.y * sc);
    h.z = f2bf(v.z * sc);
    h.w = f2bf(v.w * sc);
    *reinterpret_cast<ushort4*>(shadow + row * d + e) = h;
  }
}

struct BiasArgs {
  float* b; float* m; float* v;    // [G][n]
  const float* colpart;            // [G][tm][n] partial sums of dpre_s over row tiles
  int tm;                          // number of row tiles in colpart
  const float* enc_part;           // [G][enc_tiles][2] (l1, l0)
  int enc_tiles;
  const float* dec_part;           // [G][dec_tiles] (sum R^2)
  int dec_tiles;
  const float* cnt_part;           // optional [G][cnt_tm][n] feature on-counts
  int cnt_tm;                      // row-tile slots of cnt_part (the bias gradient may arrive reduced: tm = 1)
  float* feat_count;               // optional [G][n] accumulated counts
  const float* l1;                 // [G]
  const float* bias_decay;         // [G]
  const float* lr;                 // [G]
  float* out;                      // [G][6]: loss, l_rec, l_l1, l_bias_decay, mean L0, |b|
  int n, B, d;
  int nmodels;                     // G (the fused step tail indexes its b^2 partials by model)
  float gscale;                    // converts colpart sums to dL/db (2/(B d) for raw dpre_s)
  float b1, b2, eps, bc1, bc2;
  int update;                      // 0: only losses (eval)
  int* step;                       // optional device step counter, advanced by loss_reduce
  int defer_step;                  // 1: do not advance (the caller does, after a concurrent
                                   //    row-Adam that reads the same counter); bias Adam uses *step + 1
};

// Phase 1 (one block per model): reduce the GEMM-epilogue partials to the
// reference's loss terms and record |b| (pre-update) for the bias-decay term.
__global__ __launch_bounds__(256) void loss_reduce_kernel(BiasArgs a) {
  __shared__ float red[8];
  const int g = blockIdx.x, tid = threadIdx.x;
  const int n = a.n;
  // Only G blocks run, so every loop is latency-bound: the loads are vectorised and the loops
  // unrolled so one memory round trip serves several iterations (was ~8 us at G = 8).
  const float* b = a.b + (long)g * n;
  float bs = 0.f;
  if ((n & 3) == 0) {
    const float4* b4 = reinterpret_cast<const float4*>(b);
#pragma unroll 4
    for (int j = tid; j < n / 4; j += 256) {
      const float4 v = b4[j];
      bs += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
  } else {
#pragma unroll 4
    for (int j = tid; j < n; j += 256) bs += b[j] * b[j];
  }
  bs = block_sum_256(bs, red);
  float l1 = 0.f, l0 = 0.f, se = 0.f;
  const float2* ep = reinterpret_cast<const float2*>(a.enc_part) + (long)g * a.enc_tiles;
#pragma unroll 4
  for (int t = tid; t < a.enc_tiles; t += 256) {
    const float2 v = ep[t];
    l1 += v.x;
    l0 += v.y;
  }
#pragma unroll 4
  for (int t = tid; t < a.dec_tiles; t += 256) se += a.dec_part[(long)g * a.dec_tiles + t];
  l1 = block_sum_256(l1, red);
  l0 = block_sum_256(l0, red);
  se = block_sum_256(se, red);
  if (tid == 0) {
    const float bnorm = sqrtf(bs);
    const float l_rec = se / ((float)a.B * a.d);
    const float l_l1 = a.l1[g] * l1 / a.B;
    const float l_bd = a.bias_decay[g] * bnorm;
    float* o = a.out + g * 6;
    o[0] = l_rec + l_l1 + l_bd;
    o[1] = l_rec;
    o[2] = l_l1;
    o[3] = l_bd;
    o[4] = l0 / a.B;
    o[5] = bnorm;
    // the step counter advances once per optimizer step; bias_adam (next launch) reads the new value
    if (g == 0 && a.update && a.step && !a.defer_step) *a.step += 1;
  }
}

// Phase 2 (grid: n/32 x G, 256 threads = 8 row-groups x 32 columns): bias gradient from
// the per-row-tile column partials (each row-group sums every 8th tile, then an LDS
// reduce -- at a large gathered batch there are B/128 = 128 tiles per column), the
// bias-decay term, Adam on the bias; optional feature on-count accumulation.
__global__ __launch_bounds__(256) void bias_adam_kernel(BiasArgs a) {
  __shared__ float gred[8][33], cred[8][33];
  const int g = blockIdx.y;
  const int col = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int j = blockIdx.x * 32 + col;
  const int n = a.n;
  const bool ok = j < n;
  const bool counting = a.cnt_part && a.feat_count;
  float gs = 0.f, cs = 0.f;
  if (ok) {
    if (a.update)
      for (int t = grp; t < a.tm; t += 8) gs += a.colpart[((long)g * a.tm + t) * n + j];
    if (counting)
      for (int t = grp; t < a.cnt_tm; t += 8) cs += a.cnt_part[((long)g * a.cnt_tm + t) * n + j];
  }
  gred[grp][col] = gs;
  cred[grp][col] = cs;
  __syncthreads();
  if (grp != 0 || !ok) return;
  float gsum = 0.f, csum = 0.f;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    gsum += gred[r][col];
    csum += cred[r][col];
  }
  const long idx = (long)g * n + j;
  if (counting) a.feat_count[idx] += csum;
  if (!a.update) return;
  const float bnorm = a.out[g * 6 + 5];
  const float beta = a.bias_decay[g];
  const float bd = (beta != 0.f && bnorm > 0.f) ? beta / bnorm : 0.f;
  float bc1 = a.bc1, bc2 = a.bc2;
  if (a.step) bias_corrections(a.b1, a.b2, *a.step + a.defer_step, bc1, bc2);
  const float bj = a.b[idx];
  const float gj = gsum * a.gscale + bd * bj;
  const float mj = a.b1 * a.m[idx] + (1.f - a.b1) * gj;
  const float vj = a.b2 * a.v[idx] + (1.f - a.b2) * gj * gj;
  a.m[idx] = mj;
  a.v[idx] = vj;
  a.b[idx] = bj - (a.lr[g] / bc1) * mj / (sqrtf(vj / bc2) + a.eps);
}


// ------------------------------------------------------------------ fused step tail
// The end of a single-device training step as ONE launch (it replaces adam_rows + loss_reduce +
// bias_adam and the next step's batch-gather launch; three ~5 us latency-bound kernels and their
// launch gaps).  Block roles by index (the small latency-bound roles first, so they are not a
// tail behind the HBM-bound Adam rows):
//   [0, G)                      loss terms of model g (reduces the GEMM-epilogue partials)
//   [G, G + G n/32)             bias Adam, 32 columns of one model (+ feature on-counts)
//   [.., + rows/4)              row Adam (norm Jacobian, update, bf16 shadow, row norms)
//   [.., + ngather)             the NEXT step's batch gather from the ring permutation (last:
//                               its rows stay L2-hot for the next encoder)
// Cross-block dependencies are removed instead of ordered:
//   * |b| (loss term and bias-decay gradient, both of the pre-update bias) comes from per-32-
//     column partial sums of b^2 written by the PREVIOUS step's bias blocks (double-buffered by
//     step parity: this step reads bsq[t & 1] and writes bsq[(t + 1) & 1]);
//   * every block reads the device step counter t at its start; the last block to finish
//     (atomic ticket) advances it -- after every other block has taken its ticket, i.e. after
//     every read of t.
constexpr int TK_SUB = 64, TK_LINE = 32;  // sub-counters of the completion ticket, ints per 128-byte line

struct TailArgs {
  float* bsq;                 // [2][G][n/32] partial sums of b^2 (parity-double-buffered)
  int* ticket;                // [(1 + TK_SUB) * TK_LINE] zero-initialised counters (reset by the kernel)
  // next-step gather (ngather blocks; 0 = none): out[r] = buf[perm[(t + 1 - ep0) * rows + r]]
  const u32x4_t* gbuf; long nbuf; const long* perm; long nperm; const int* ep0; u32x4_t* gout; long grows;
  int row_vec;
  int nloss, nbias, ngather;  // block counts of the roles
  // masked ensembles: the row-Adam blocks cover only live rows (lcomp: live-row prefix lpre[g] over
  // the models, the same for every set; compact row rc of set s -> row g n + rc - lpre[g] of model g)
  int lcomp, lG, lpre[17];
  // top-k step tail (sc_topk_tail): the loss blocks reduce per-row squared errors instead of the SAE
  // epilogue partials -- mse[g] = se_scale * sum_r row_se[g][r]; no bias blocks
  const float* row_se; int se_rows; float se_scale; float* mse;
};

__device__ __forceinline__ void tail_loss(const BiasArgs& a, const TailArgs& t, int g, int par) {
  __shared__ float red[8];
  const int tid = threadIdx.x, nb = a.n / 32;
  float bs = 0.f;
  for (int j = tid; j < nb; j += 256) bs += t.bsq[((long)par * a.nmodels + g) * nb + j];
  bs = block_sum_256(bs, red);
  float l1 = 0.f, l0 = 0.f, se = 0.f;
  const float2* ep = reinterpret_cast<const float2*>(a.enc_part) + (long)g * a.enc_tiles;
#pragma unroll 4
  for (int k = tid; k < a.enc_tiles; k += 256) {
    const float2 v = ep[k];
    l1 += v.x;
    l0 += v.y;
  }
#pragma unroll 4
  for (int k = tid; k < a.dec_tiles; k += 256) se += a.dec_part[(long)g * a.dec_tiles + k];
  l1 = block_sum_256(l1, red);
  l0 = block_sum_256(l0, red);
  se = block_sum_256(se, red);
  if (tid == 0) {
    const float bnorm = sqrtf(bs);
    const float l_rec = se / ((float)a.B * a.d);
    const float l_l1 = a.l1[g] * l1 / a.B;
    const float l_bd = a.bias_decay[g] * bnorm;
    float* o = a.out + g * 6;
    o[0] = l_rec + l_l1 + l_bd;
    o[1] = l_rec;
    o[2] = l_l1;
    o[3] = l_bd;
    o[4] = l0 / a.B;
    o[5] = bnorm;
  }
}

__device__ __forceinline__ void tail_mse(const TailArgs& t, int g) {
  __shared__ float red[8];
  float se = 0.f;
  const float* rs = t.row_se + (long)g * t.se_rows;
#pragma unroll 4
  for (int r = threadIdx.x; r < t.se_rows; r += 256) se += rs[r];
  se = block_sum_256(se, red);
  if (threadIdx.x == 0) t.mse[g] = se * t.se_scale;
}

__device__ __forceinline__ void tail_bias(const BiasArgs& a, const TailArgs& t, int bx, int g, int step, int par) {
  __shared__ float gred[8][33], cred[8][33], sred[8];
  const int col = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int n = a.n, nb = n / 32;
  const int j = bx * 32 + col;
  const bool counting = a.cnt_part && a.feat_count;
  // |b| of the pre-update bias from the previous step's partials (every block of the model alike)
  float bs = 0.f;
  for (int k = threadIdx.x; k < nb; k += 256) bs += t.bsq[((long)par * a.nmodels + g) * nb + k];
  bs = block_sum_256(bs, sred);
  float gs = 0.f, cs = 0.f;
  for (int k = grp; k < a.tm; k += 8) gs += a.colpart[((long)g * a.tm + k) * n + j];
  // (on-counts keep the encoder's 128-row slots even when the bias gradient arrives reduced, tm = 1)
  if (counting)
    for (int k = grp; k < a.cnt_tm; k += 8) cs += a.cnt_part[((long)g * a.cnt_tm + k) * n + j];
  gred[grp][col] = gs;
  cred[grp][col] = cs;
  __syncthreads();
  if (grp != 0) return;
  float gsum = 0.f, csum = 0.f;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    gsum += gred[r][col];
    csum += cred[r][col];
  }
  const long idx = (long)g * n + j;
  if (counting) a.feat_count[idx] += csum;
  const float bnorm = sqrtf(bs);
  const float beta = a.bias_decay[g];
  const float bd = (beta != 0.f && bnorm > 0.f) ? beta / bnorm : 0.f;
  float bc1, bc2;
  bias_corrections(a.b1, a.b2, step + 1, bc1, bc2);
  const float bj = a.b[idx];
  const float gj = gsum * a.gscale + bd * bj;
  const float mj = a.b1 * a.m[idx] + (1.f - a.b1) * gj;
  const float vj = a.b2 * a.v[idx] + (1.f - a.b2) * gj * gj;
  a.m[idx] = mj;
  a.v[idx] = vj;
  const float bn = bj - (a.lr[g] / bc1) * mj / (sqrtf(vj / bc2) + a.eps);
  a.b[idx] = bn;
  // this block's 32 columns of |b_new|^2 for the next step (lanes 0-31 of wave 0)
  float sq = bn * bn;
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 32);
  if (col == 0) t.bsq[((long)(par ^ 1) * a.nmodels + g) * nb + bx] = sq;
}

template <int NV, bool GBF>
__global__ __launch_bounds__(256) void step_tail_kernel(AdamArgs a, BiasArgs b, TailArgs t) {
  const int bid = blockIdx.x;
  const int step = *a.step;          // completed steps before this one (t); read by every block
  const int par = step & 1;
  if (bid < t.nloss) {
    if (t.row_se) tail_mse(t, bid);
    else tail_loss(b, t, bid, par);
  } else if (bid < t.nloss + t.nbias) {
    const int k = bid - t.nloss, nb = b.n / 32;
    tail_bias(b, t, k % nb, k / nb, step, par);
  } else if (bid >= (int)gridDim.x - t.ngather) {
    // the next step's batch: the LAST blocks dispatched, so the rows are written at the end of the
    // launch and still sit in L2 when the next step's encoder reads them (written first, the Adam
    // stream evicted them: encoder 67 vs 57 us, measured)
    const long r = (long)(bid - ((int)gridDim.x - t.ngather)) * 4 + (threadIdx.x >> 6);
    if (r < t.grows) {
      const int lane = threadIdx.x & 63;
      const long jj = (long)(step + 1 - t.ep0[0]) * t.grows + r;
      long src = (jj >= 0 && jj < t.nperm) ? t.perm[jj] : 0;
      src = (src >= 0 && src < t.nbuf) ? src : 0;
      const u32x4_t* sp = t.gbuf + src * t.row_vec;
      u32x4_t* op = t.gout + r * t.row_vec;
      for (int v = lane; v < t.row_vec; v += 64) op[v] = sp[v];
    }
  } else {
    long r = (long)(bid - t.nloss - t.nbias) * 4 + (threadIdx.x >> 6);
    if (t.lcomp) {  // compacted masked grid: skip the dead rows' blocks altogether
      const long per = t.lpre[t.lG];
      const int s = (int)(r / per);
      long rc = r - s * per;
      int g = 0;
#pragma unroll
      for (int k = 1; k < 16; ++k)
        if (k < t.lG && rc >= t.lpre[k]) g = k;
      r = s < a.nset ? (long)s * a.set[0].rows + (long)g * a.rows_per_model + (rc - t.lpre[g]) : a.set[0].rows * 2;
    }
    adam_row<NV, GBF>(a, r);
  }
  // The last block to finish advances the step counter.  Every block's read of *step was consumed
  // (bias corrections, parity) before its ticket, so no fence is needed -- and none is wanted: an
  // agent-scope release writes back the XCD's L2 (one per block: ~2.4x the whole step, measured).
  // Relaxed agent-scope RMWs are coherent across the XCDs.  The tickets are two-level: one RMW
  // per block on one of TK_SUB counters (each on its own 128-byte line, so the ~9k RMWs spread
  // over many L2 channels instead of serialising on one address: +33 us per step, measured),
  // and the block completing a sub-counter takes a ticket on the top counter.
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nb = (int)gridDim.x, sub = bid % TK_SUB;
    const int expect = nb / TK_SUB + (sub < nb % TK_SUB ? 1 : 0);
    int* sc = t.ticket + (1 + sub) * TK_LINE;
    if (__hip_atomic_fetch_add(sc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == expect - 1) {
      __hip_atomic_store(sc, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int nsub = nb < TK_SUB ? nb : TK_SUB;
      if (__hip_atomic_fetch_add(t.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsub - 1) {
        __hip_atomic_store(t.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(b.step, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

}  // namespace scamd

using namespace scamd;

extern "C" {

int sc_adam_rows(int nset, float* const* p, const void* const* g, float* const* m, float* const* v,
                 void* const* shadow, float* const* norms, const int* rows, const int* norm, int d,
                 int rows_per_model, const float* lr, float b1, float b2, float eps, float bc1,
                 float bc2, const int* step, int nsplit, long gstride, long row0, hipStream_t stream,
                 const int* live, int gbf16) {
  if (d % 256 || d > 4096 || nset < 1 || nset > 2 || nsplit < 1) return 1;
  AdamArgs a;
  long total = 0;
  for (int i = 0; i < nset; ++i) {
    a.set[i] = {p[i], g[i], m[i], v[i], reinterpret_cast<uint16_t*>(shadow[i]), norms[i], rows[i], norm[i]};
    total += rows[i];
  }
  if (nset == 1) a.set[1] = a.set[0], a.set[1].rows = 0;
  a.nset = nset; a.d = d; a.rows_per_model = rows_per_model; a.lr = lr;
  a.b1 = b1; a.b2 = b2; a.eps = eps; a.bc1 = bc1; a.bc2 = bc2; a.step = step;
  a.nsplit = nsplit; a.gstride = gstride; a.row0 = row0; a.live = live;
  const long blocks = (total + 3) / 4;
  // bf16 gradients: plain loads only (the NT knob A/B'd slower, profiles/)
#define SC_ADAM(NVV)                                                                                  \
  case NVV:                                                                                           \
    if (gbf16) hipLaunchKernelGGL((adam_rows_kernel<NVV, true>), dim3(blocks), dim3(256), 0, stream, a); \
    else hipLaunchKernelGGL((adam_rows_kernel<NVV>), dim3(blocks), dim3(256), 0, stream, a);            \
    break;
  switch (d / 256) {
    SC_ADAM(1) SC_ADAM(2) SC_ADAM(3) SC_ADAM(4) SC_ADAM(6) SC_ADAM(8) SC_ADAM(16)
    default: return 1;
  }
#undef SC_ADAM
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int sc_shadow_rows(const float* p, void* shadow, float* norms, long rows, int d, int norm,
                   hipStream_t stream) {
  if (d % 4) return 1;
  hipLaunchKernelGGL(shadow_rows_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, p,
                     reinterpret_cast<uint16_t*>(shadow), norms, rows, d, norm);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int sc_bias_loss(int G, float* b, float* m, float* v, const float* colpart, int tm,
                 const float* enc_part, int enc_tiles, const float* dec_part, int dec_tiles,
                 const float* cnt_part, float* feat_count, const float* l1, const float* bias_decay,
                 const float* lr, float* out, int n, int B, int d, float gscale, float b1, float b2, float eps,
                 float bc1, float bc2, int update, int* step, hipStream_t stream, int defer_step, int cnt_tm) {
  BiasArgs a;
  a.b = b; a.m = m; a.v = v; a.colpart = colpart; a.tm = tm;
  a.enc_part = enc_part; a.enc_tiles = enc_tiles; a.dec_part = dec_part; a.dec_tiles = dec_tiles;
  a.cnt_part = cnt_part; a.feat_count = feat_count; a.cnt_tm = cnt_tm > 0 ? cnt_tm : tm;
  a.l1 = l1; a.bias_decay = bias_decay; a.lr = lr; a.out = out;
  a.n = n; a.B = B; a.d = d; a.nmodels = G; a.gscale = gscale;
  a.b1 = b1; a.b2 = b2; a.eps = eps; a.bc1 = bc1; a.bc2 = bc2; a.update = update; a.step = step;
  a.defer_step = defer_step ? 1 : 0;
  hipLaunchKernelGGL(loss_reduce_kernel, dim3(G), dim3(256), 0, stream, a);
  if (update || (cnt_part && feat_count))
    hipLaunchKernelGGL(bias_adam_kernel, dim3((n + 31) / 32, G), dim3(256), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// Fused step tail (see step_tail_kernel): row Adam over the sets + loss terms + bias Adam, the next
// step's batch gather when gbuf != nullptr, and the device step counter advanced by the last block.
// bsq: [2][G][n/32] b^2 partials (parity of *step current); ticket: one zero-initialised int.
int sc_step_tail(int nset, float* const* p, const void* const* g, float* const* m, float* const* v,
                 void* const* shadow, float* const* norms, const int* rows, const int* norm, int d,
                 int rows_per_model, const float* lr, float b1, float b2, float eps, int* step, int gbf16,
                 int G, float* b, float* bm, float* bv, const float* colpart, int tm, const float* enc_part,
                 int enc_tiles, const float* dec_part, int dec_tiles, const float* cnt_part, float* feat_count,
                 const float* l1, const float* bias_decay, float* out, int n, int B, float gscale,
                 float* bsq, int* ticket, const void* gbuf, long nbuf, const long* perm, long nperm,
                 const int* ep0, void* gout, long grows, long row_bytes, int nsplit, long gstride,
                 const int* live, int cnt_tm, long row0, const int* live_h, hipStream_t stream) {
  if (d % 256 || d > 4096 || nset < 1 || nset > 2 || n % 32 || !step || !ticket || !bsq || nsplit < 1) return 1;
  if (gbuf && (row_bytes % 16 || nbuf < 1)) return 1;
  AdamArgs a;
  long total = 0;
  for (int i = 0; i < nset; ++i) {
    a.set[i] = {p[i], g[i], m[i], v[i], reinterpret_cast<uint16_t*>(shadow[i]), norms[i], rows[i], norm[i]};
    total += rows[i];
  }
  if (nset == 1) a.set[1] = a.set[0], a.set[1].rows = 0;
  a.nset = nset; a.d = d; a.rows_per_model = rows_per_model; a.lr = lr;
  a.b1 = b1; a.b2 = b2; a.eps = eps; a.bc1 = 1.f; a.bc2 = 1.f; a.step = step;
  // live: masked ensembles (may be null); row0: the sets are rows [row0, row0 + rows) of the
  // [G n] stack (a ZeRO-1 shard; the loss and bias roles still cover every model)
  a.nsplit = nsplit; a.gstride = gstride; a.row0 = row0; a.live = live;
  BiasArgs ba;
  ba.b = b; ba.m = bm; ba.v = bv; ba.colpart = colpart; ba.tm = tm;
  ba.enc_part = enc_part; ba.enc_tiles = enc_tiles; ba.dec_part = dec_part; ba.dec_tiles = dec_tiles;
  // (the bias gradient may arrive reduced -- data parallel: tm = 1 -- while the on-counts keep the
  // encoder's per-128-row slots)
  ba.cnt_part = cnt_part; ba.feat_count = feat_count; ba.cnt_tm = cnt_tm > 0 ? cnt_tm : tm;
  ba.l1 = l1; ba.bias_decay = bias_decay; ba.lr = lr; ba.out = out;
  ba.n = n; ba.B = B; ba.d = d; ba.nmodels = G; ba.gscale = gscale;
  ba.b1 = b1; ba.b2 = b2; ba.eps = eps; ba.bc1 = 1.f; ba.bc2 = 1.f; ba.update = 1; ba.step = step;
  ba.defer_step = 0;
  TailArgs t;
  t.bsq = bsq; t.ticket = ticket;
  t.gbuf = reinterpret_cast<const u32x4_t*>(gbuf); t.nbuf = nbuf; t.perm = perm; t.nperm = nperm; t.ep0 = ep0;
  t.gout = reinterpret_cast<u32x4_t*>(gout); t.grows = gbuf ? grows : 0;
  t.row_vec = (int)(row_bytes / 16);
  t.nloss = G; t.nbias = G * (n / 32); t.ngather = gbuf ? (int)((grows + 3) / 4) : 0;
  t.lcomp = 0; t.lG = G;
  t.row_se = nullptr; t.se_rows = 0; t.se_scale = 0.f; t.mse = nullptr;
  long arows = total;
  // host copy of a masked ensemble's live sizes (full-stack sets only, G <= 16): launch live rows only
  if (live_h && live && row0 == 0 && G <= 16 && rows_per_model > 0 && rows[0] == (long)G * rows_per_model &&
      (nset == 1 || rows[1] == rows[0])) {
    t.lpre[0] = 0;
    for (int g = 0; g < G; ++g)
      t.lpre[g + 1] = t.lpre[g] + std::min(rows_per_model, std::max(0, live_h[g]));
    for (int g = G + 1; g < 17; ++g) t.lpre[g] = t.lpre[G];
    if (t.lpre[G] > 0) {
      t.lcomp = 1;
      arows = (long)nset * t.lpre[G];
    }
  }
  const long blocks = t.nloss + t.nbias + t.ngather + (arows + 3) / 4;
#define SC_TAIL(NVV)                                                                                   \
  case NVV:                                                                                            \
    if (gbf16) hipLaunchKernelGGL((step_tail_kernel<NVV, true>), dim3(blocks), dim3(256), 0, stream, a, ba, t); \
    else hipLaunchKernelGGL((step_tail_kernel<NVV, false>), dim3(blocks), dim3(256), 0, stream, a, ba, t);      \
    break;
  switch (d / 256) {
    SC_TAIL(1) SC_TAIL(2) SC_TAIL(3) SC_TAIL(4)
    default: return 1;
  }
#undef SC_TAIL
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// Top-k step tail (engine/topk.py): row Adam with the norm Jacobian over the [G n, d] dictionary stack
// + the per-model MSE from the decode's per-row squared errors (mse[g] = se_scale sum_r row_se[g][r])
// + the next step's batch gather (gbuf != nullptr), and the device step counter advanced by the last
// block: one launch instead of Adam + two torch reductions + the counter increment + a gather.
int sc_topk_tail(float* p, const void* g, float* m, float* v, void* shadow, float* norms, int G, int n, int d,
                 const float* lr, float b1, float b2, float eps, int* step, int gbf16, const float* row_se,
                 int se_rows, float se_scale, float* mse, int* ticket, const void* gbuf, long nbuf,
                 const long* perm, long nperm, const int* ep0, void* gout, long grows, long row_bytes,
                 hipStream_t stream) {
  if (d % 256 || d > 1024 || G < 1 || n < 1 || !step || !ticket || !row_se || !mse || se_rows < 1) return 1;
  if (gbuf && (row_bytes % 16 || nbuf < 1)) return 1;
  AdamArgs a;
  a.set[0] = {p, g, m, v, reinterpret_cast<uint16_t*>(shadow), norms, G * n, 1};
  a.set[1] = a.set[0];
  a.set[1].rows = 0;
  a.nset = 1; a.d = d; a.rows_per_model = n; a.lr = lr;
  a.b1 = b1; a.b2 = b2; a.eps = eps; a.bc1 = 1.f; a.bc2 = 1.f; a.step = step;
  a.nsplit = 1; a.gstride = 0; a.row0 = 0; a.live = nullptr;
  BiasArgs ba = {};
  ba.step = step; ba.nmodels = G; ba.n = n;
  TailArgs t = {};
  t.ticket = ticket;
  t.gbuf = reinterpret_cast<const u32x4_t*>(gbuf); t.nbuf = nbuf; t.perm = perm; t.nperm = nperm; t.ep0 = ep0;
  t.gout = reinterpret_cast<u32x4_t*>(gout); t.grows = gbuf ? grows : 0;
  t.row_vec = (int)(row_bytes / 16);
  t.nloss = G; t.nbias = 0; t.ngather = gbuf ? (int)((grows + 3) / 4) : 0;
  t.lcomp = 0; t.lG = G;
  t.row_se = row_se; t.se_rows = se_rows; t.se_scale = se_scale; t.mse = mse;
  const long blocks = t.nloss + t.ngather + ((long)G * n + 3) / 4;
#define SC_TAIL(NVV)                                                                                   \
  case NVV:                                                                                            \
    if (gbf16) hipLaunchKernelGGL((step_tail_kernel<NVV, true>), dim3(blocks), dim3(256), 0, stream, a, ba, t); \
    else hipLaunchKernelGGL((step_tail_kernel<NVV, false>), dim3(blocks), dim3(256), 0, stream, a, ba, t);      \
    break;
  switch (d / 256) {
    SC_TAIL(1) SC_TAIL(2) SC_TAIL(3) SC_TAIL(4)
    default: return 1;
  }
#undef SC_TAIL
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
