// Top-k sparse coding kernels for an ensemble with per-model k (gfx950).
//
// Reference: TopKEncoder (autoencoders/topk_encoder.py:19-40): scores = x D^T,
// keep each row's top-k, ReLU, x_hat = code D, MSE.  The reference cannot
// vmap over models because k changes the output shape (no_stacking=True,
// big_sweep_experiments.py:246-253); here k lives in device memory and every
// model runs in the same launches:
//   topk_select_kernel   : exact per-row radix select (11/11/10-bit passes over the
//                          orderable bit pattern, per-wave LDS histograms, parallel
//                          digit search), scores kept in registers; emits (idx, value)
//                          pairs in column order.
//   topk_decode_grad     : one wave per row: sparse decode x_hat = sum_j v_j D[idx_j]
//                          (bf16 dictionary gathered from L2), residual, per-row
//                          squared error, then the k code gradients <R, D[idx_j]>
//                          scattered into dense bf16 buffers for the MFMA wgrad GEMM.
//   topk_clear           : zeroes exactly the scattered positions afterwards.
#include "common.h"
#include <stdlib.h>

namespace scamd {

__device__ __forceinline__ uint32_t order_key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // larger float -> larger key
}

// Exact per-row top-k by radix select on the orderable bit pattern: three digit
// passes (11, 11, 10 bits).  Each pass builds the histogram of the still-eligible
// keys in four per-wave copies (a quarter of the LDS-atomic contention of one
// shared histogram: the leading digit of similar-magnitude scores hits few bins),
// then all 256 threads locate the digit holding the k-th largest key with a
// block-wide suffix scan (no serial bin walk).  Selected entries are written in a
// fixed thread-major order from one packed block scan, ties at the threshold are
// taken in that order, so the output is deterministic.
constexpr int TK_NT = 256;
constexpr int TK_BINS = 2048;

template <int PER>  // keys per thread (n <= 256 * PER)
__global__ __launch_bounds__(TK_NT, 4) void topk_select_kernel(const float* __restrict__ scores, const int* __restrict__ kv,
                                                            int* __restrict__ idx, float* __restrict__ val, int B, int n,
                                                            int kmax, int absolute, int relu) {
  __shared__ uint32_t hist[4][TK_BINS];
  __shared__ uint32_t wsum[8];
  __shared__ int sel[2];  // selected digit, keys strictly above it
  const long row = blockIdx.x;
  const int g = row / B;
  const int k = min(kv[g], n);
  const float* S = scores + row * n;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t key[PER];
  float sv[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = tid + i * TK_NT;
    const float s = S[min(c, n - 1)];  // unconditional load + branch-free mask (see topk_wave_kernel)
    sv[i] = s;
    key[i] = order_key(absolute ? fabsf(s) : s) & (0u - (uint32_t)(c < n));  // padding sorts below every key
  }
  uint32_t prefix = 0, mask = 0;
  int remaining = k;
  const int shifts[3] = {21, 10, 0};
  const int widths[3] = {11, 11, 10};
#pragma unroll
  for (int pass = 0; pass < 3; ++pass) {
    if (k == 0) break;
    const int shift = shifts[pass];
    const uint32_t dmask = (1u << widths[pass]) - 1u;
    for (int b = tid; b < 4 * TK_BINS; b += TK_NT) (&hist[0][0])[b] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if (tid + i * TK_NT < n && (key[i] & mask) == prefix) atomicAdd(&hist[w][(key[i] >> shift) & dmask], 1u);
    }
    __syncthreads();
    // thread t owns bins [8t, 8t + 8) (descending search: high bins first)
    uint32_t cnt[8], tot = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int b = tid * 8 + j;
      cnt[j] = hist[0][b] + hist[1][b] + hist[2][b] + hist[3][b];
      tot += cnt[j];
    }
    // suffix sum over threads: above(t) = sum of totals of threads > t
    uint32_t incl = tot;  // inclusive suffix scan within the wave (lanes above)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_down(incl, o, 64);
      if (lane + o < 64) incl += v;
    }
    if (lane == 0) wsum[w] = incl;  // wave total
    __syncthreads();
    uint32_t above = incl - tot;  // lanes above within the wave
    for (int ww = w + 1; ww < 4; ++ww) above += wsum[ww];
    // the k-th largest key lies in this thread's range iff above < remaining <= above + tot
    if (above < (uint32_t)remaining && (uint32_t)remaining <= above + tot) {
      uint32_t a = above;
      int j = 7;
      for (; j > 0; --j) {
        if (a + cnt[j] >= (uint32_t)remaining) break;
        a += cnt[j];
      }
      sel[0] = tid * 8 + j;
      sel[1] = (int)a;
    }
    __syncthreads();
    prefix |= (uint32_t)sel[0] << shift;
    mask |= dmask << shift;
    remaining -= sel[1];
    __syncthreads();
  }
  // prefix is the k-th largest key: take every key above it and the first `remaining`
  // ties.  Output order is thread-major (thread t's keys in i order, then thread t+1):
  // deterministic, one block-wide scan of packed (above, tie) counts.
  int* I = idx + row * kmax;
  float* V = val + row * kmax;
  if (k > 0) {
    uint32_t na = 0, nt = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const bool valid = tid + i * TK_NT < n;
      na += (valid && key[i] > prefix) ? 1u : 0u;
      nt += (valid && key[i] == prefix) ? 1u : 0u;
    }
    const uint32_t packed = (na << 16) | nt;  // n <= 65535
    uint32_t incl = packed;  // inclusive prefix within the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t excl = incl - packed;
    for (int ww = 0; ww < w; ++ww) excl += wsum[ww];
    int pos_a = (int)(excl >> 16);          // keys above the threshold before this thread
    int tie_rank = (int)(excl & 0xFFFFu);   // ties before this thread
    // taken ties occupy the slots after every key above; keys above come first in slot order
    uint32_t tot = 0;
    for (int ww = 0; ww < 4; ++ww) tot += wsum[ww];
    const int total_above = (int)(tot >> 16);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * TK_NT;
      if (c >= n) continue;
      int pos = -1;
      if (key[i] > prefix) {
        pos = pos_a++;
      } else if (key[i] == prefix) {
        if (tie_rank < remaining) pos = total_above + tie_rank;
        ++tie_rank;
      }
      if (pos >= 0) {
        I[pos] = c;
        V[pos] = relu ? fmaxf(sv[i], 0.f) : sv[i];
      }
    }
  }
  // pad the unused slots of models with k < kmax
  for (int j = k + tid; j < kmax; j += TK_NT) {
    I[j] = 0;
    V[j] = 0.f;
  }
}

// ---------------------------------------------------------------------------
// Wave-per-row exact top-k (n <= 64 * PL): the row's keys live in one wave's VGPRs,
// so there is no LDS histogram, no atomics and no block barrier (the radix kernel
// above pays 3 x (histogram clear, bank-conflicted LDS atomics, scan) behind 256-thread
// barriers).  Every count is a ballot + scalar popcount: one v_cmp per key and no
// cross-lane reduction latency.  The k-th largest key T is found by bisection on its
// bits (MSB first: t | bit is kept iff count(key >= t | bit) >= k).  The first S1 = 12
// bits scan all keys; then the keys sharing t's top 12 bits (the "bucket", a handful
// for score rows) are compacted one per lane and each remaining bit costs one ballot.
// Output: every key > T and the first (k - count(> T)) keys == T, in column order.
// Wave-wide integer sum on the DPP path (row scans + row broadcasts, then lane 63):
// six VALU adds and a readlane instead of ds_bpermute round trips or a per-key ballot +
// scalar popcount chain (the CU's one scalar unit serialises those across its waves).
__device__ __forceinline__ int wave_total(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ int lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

template <int PL>
__global__ __launch_bounds__(256) void topk_wave_kernel(const float* __restrict__ scores, const int* __restrict__ kv,
                                                      int* __restrict__ idx, float* __restrict__ val, long rows, int B,
                                                      int n, int kmax, int absolute, int relu) {
  constexpr int S1 = 12;            // full-scan bisection steps before compaction
  constexpr int LOW = 32 - S1;      // bits resolved on the compacted bucket
  __shared__ uint32_t cbuf[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long row = (long)blockIdx.x * 4 + w;
  if (row >= rows) return;          // per-wave work only: no block barrier below
  const int g = (int)(row / B);
  const int k = min(kv[g], n);
  const float* S = reinterpret_cast<const float*>(__builtin_assume_aligned(scores + row * n, 16));
  int* I = idx + row * kmax;
  float* V = val + row * kmax;
  uint32_t key[PL];
#pragma unroll
  for (int i = 0; i < PL / 4; ++i) {
    const int c = (i * 64 + lane) * 4;
    // unconditional (clamped, 16-byte aligned: n % 4 == 0) loads and a branch-free mask: a
    // guarded load or key makes hipcc branch and wait vmcnt(0) per load, serialising them
    const float4 v = *reinterpret_cast<const float4*>(
        __builtin_assume_aligned(S + (min(c, n - 4) & ~3), 16));
    const uint32_t live = 0u - (uint32_t)(c < n);
    const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) key[4 * i + j] = order_key(absolute ? fabsf(f[j]) : f[j]) & live;
  }
  if (k > 0) {
    uint32_t t = 0;
#pragma unroll 1
    for (int b = 31; b >= LOW; --b) {
      const uint32_t cand = t | (1u << b);
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < PL; ++i) cnt += key[i] >= cand ? 1 : 0;
      if (wave_total(cnt) >= k) t = cand;
    }
    const uint32_t hi = t >> LOW;
    int above = 0, inb = 0;
#pragma unroll
    for (int i = 0; i < PL; ++i) {
      const uint32_t h = key[i] >> LOW;
      above += h > hi ? 1 : 0;
      inb += h == hi ? 1 : 0;
    }
    const int n_above = wave_total(above), nb = wave_total(inb);
    int gt;
    if (nb <= 64) {
      // lane offsets: exclusive scan of the per-lane bucket counts (DPP row scan + row
      // totals through lanes 15/31/47), then each lane writes its own bucket keys
      int incl = inb;
      incl += __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xf, 0xf, false);
      incl += __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xf, 0xf, false);
      incl += __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xf, 0xf, false);
      incl += __builtin_amdgcn_update_dpp(0, incl, 0x118, 0xf, 0xf, false);
      const int r0 = __builtin_amdgcn_readlane(incl, 15), r1 = __builtin_amdgcn_readlane(incl, 31);
      const int r2 = __builtin_amdgcn_readlane(incl, 47);
      const int rowoff = lane < 16 ? 0 : lane < 32 ? r0 : lane < 48 ? r0 + r1 : r0 + r1 + r2;
      int off = rowoff + incl - inb;
#pragma unroll
      for (int i = 0; i < PL; ++i)
        if ((key[i] >> LOW) == hi) cbuf[w][off++] = key[i];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const bool valid = lane < nb;
      const uint32_t ck = valid ? cbuf[w][lane] : 0u;
#pragma unroll 1
      for (int b = LOW - 1; b >= 0; --b) {
        const uint32_t cand = t | (1u << b);
        if (n_above + __popcll(__ballot(valid && ck >= cand)) >= k) t = cand;
      }
      gt = n_above + __popcll(__ballot(valid && ck > t));
    } else {  // a crowded bucket (many equal / near-equal scores): finish by full scans
#pragma unroll 1
      for (int b = LOW - 1; b >= 0; --b) {
        const uint32_t cand = t | (1u << b);
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < PL; ++i) cnt += key[i] >= cand ? 1 : 0;
        if (wave_total(cnt) >= k) t = cand;
      }
      int c2 = 0;
#pragma unroll
      for (int i = 0; i < PL; ++i) c2 += key[i] > t ? 1 : 0;
      gt = wave_total(c2);
    }
    const int need_ties = k - gt;
    // output in column order: chunk i covers columns [256 i, 256 i + 256), lane l owns
    // columns 256 i + 4 l + j (j < 4), so column order = (lane, j) within a chunk
    int base = 0, ties_seen = 0;
#pragma unroll
    for (int i = 0; i < PL / 4; ++i) {
      uint64_t me[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) me[j] = __ballot(key[4 * i + j] == t);
      int tie_rank = ties_seen;  // ties in earlier columns of the row
#pragma unroll
      for (int j = 0; j < 4; ++j) tie_rank += lanes_below(me[j]);
      bool take[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t kk = key[4 * i + j];
        take[j] = kk > t || (kk == t && tie_rank < need_ties);
        tie_rank += kk == t ? 1 : 0;
      }
      uint64_t mt[4];
      int pos = base, tot = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        mt[j] = __ballot(take[j]);
        pos += lanes_below(mt[j]);
        tot += __popcll(mt[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (take[j]) {
          const int c = (i * 64 + lane) * 4 + j;
          const float sv = S[c];
          I[pos] = c;
          V[pos] = relu ? fmaxf(sv, 0.f) : sv;
          ++pos;
        }
      }
      base += tot;
#pragma unroll
      for (int j = 0; j < 4; ++j) ties_seen += __popcll(me[j]);
    }
  }
  for (int j = k + lane; j < kmax; j += 64) {
    I[j] = 0;
    V[j] = 0.f;
  }
}

// ---------------------------------------------------------------------------
// Block-per-row bisection for long rows (4096 < n <= 256 * PL): the same algorithm as
// topk_wave_kernel with the row spread over 4 waves (PL keys per thread), so every
// full-scan step costs PL compares per lane plus a DPP wave total and one LDS exchange
// (parity-double-buffered slots: one barrier per step).  After S1 = 12 bits the bucket
// (keys sharing t's top bits) is compacted into LDS and -- when it holds <= 64 keys,
// the usual case -- wave 0 resolves the last 20 bits with ballots alone.
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
  const int r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31);
  const int r2 = __builtin_amdgcn_readlane(v, 47);
  return v + (lane < 16 ? 0 : lane < 32 ? r0 : lane < 48 ? r0 + r1 : r0 + r1 + r2);
}

// Bracketed select (k <= 256): the k-th largest of the 256 per-thread maxima is a lower
// bound lo of the row's k-th largest key (at least k keys reach it), and for score rows only
// ~k .. 1.4k keys do, so ONE full pass compacts the candidates >= lo into LDS and wave 0
// bisects the handful of candidates with ballots -- instead of 12 full-row bisection passes
// (the old path was VALU-bound: 2 ops per key per pass; measured 204 -> 119 us on config 4).
// Returns false (block-uniform) when more than BR_CAP keys reach lo (heavy ties, e.g. an
// all-zero row); the caller then runs the full bisection.  Output order: thread-major
// (thread, chunk, j), deterministic; ties at the threshold are taken in that order.
constexpr int BR_CAP = 1024;

template <int PL>
__device__ __forceinline__ bool bracket_select(const uint32_t (&key)[PL], int k, int tid, int lane, int w,
                                               const float* S, int* I, float* V, int relu, uint32_t* mx,
                                               uint32_t* ckey, int* ccol, int* wsum, uint32_t* sres) {
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < PL; ++i) m = max(m, key[i]);
  mx[tid] = m;
  __syncthreads();
  if (w == 0) {
    const uint32_t a0 = mx[lane], a1 = mx[lane + 64], a2 = mx[lane + 128], a3 = mx[lane + 192];
    uint32_t t = 0;
#pragma unroll 1
    for (int b = 31; b >= 0; --b) {
      const uint32_t cand = t | (1u << b);
      const int cnt = __popcll(__ballot(a0 >= cand)) + __popcll(__ballot(a1 >= cand)) +
                      __popcll(__ballot(a2 >= cand)) + __popcll(__ballot(a3 >= cand));
      if (cnt >= k) t = cand;
    }
    if (lane == 0) sres[0] = t;
  }
  __syncthreads();
  const uint32_t lo = sres[0];
  int c = 0;
#pragma unroll
  for (int i = 0; i < PL; ++i) c += key[i] >= lo ? 1 : 0;
  const int incl = wave_incl_scan(c, lane);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int off = incl - c, total = 0;
#pragma unroll
  for (int ww = 0; ww < 4; ++ww) {
    if (ww < w) off += wsum[ww];
    total += wsum[ww];
  }
  if (total > BR_CAP) return false;
#pragma unroll
  for (int i = 0; i < PL / 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (key[4 * i + j] >= lo) {
        ckey[off] = key[4 * i + j];
        ccol[off] = (i * 256 + tid) * 4 + j;
        ++off;
      }
  __syncthreads();
  if (w == 0) {
    const int nq = (total + 63) >> 6;
    uint32_t ck[BR_CAP / 64];
#pragma unroll
    for (int q = 0; q < BR_CAP / 64; ++q) ck[q] = (q < nq && q * 64 + lane < total) ? ckey[q * 64 + lane] : 0u;
    uint32_t t = 0;
#pragma unroll 1
    for (int b = 31; b >= 0; --b) {
      const uint32_t cand = t | (1u << b);
      int cnt = 0;
#pragma unroll
      for (int q = 0; q < BR_CAP / 64; ++q)
        if (q < nq) cnt += __popcll(__ballot(ck[q] >= cand));
      if (cnt >= k) t = cand;
    }
    int gt = 0;
#pragma unroll
    for (int q = 0; q < BR_CAP / 64; ++q)
      if (q < nq) gt += __popcll(__ballot(ck[q] > t));
    const int need = k - gt;
    int base = 0, ties = 0;
#pragma unroll
    for (int q = 0; q < BR_CAP / 64; ++q) {
      if (q < nq) {
        const uint32_t kk = ck[q];
        const bool eq = kk == t && q * 64 + lane < total;
        const uint64_t me = __ballot(eq);
        const bool take = kk > t || (eq && ties + lanes_below(me) < need);
        const uint64_t mt = __ballot(take);
        if (take) {
          const int pos = base + lanes_below(mt);
          const int col = ccol[q * 64 + lane];
          const float sv = S[col];
          I[pos] = col;
          V[pos] = relu ? fmaxf(sv, 0.f) : sv;
        }
        base += __popcll(mt);
        ties += __popcll(me);
      }
    }
  }
  return true;
}

template <int PL>
__global__ __launch_bounds__(256) void topk_block_kernel(const float* __restrict__ scores, const int* __restrict__ kv,
                                                       int* __restrict__ idx, float* __restrict__ val, int B, int n,
                                                       int kmax, int absolute, int relu, int bracket) {
  constexpr int S1 = 12, LOW = 32 - S1;
  __shared__ int red[2][4];
  __shared__ int wsum[2][4];
  __shared__ uint32_t cbuf[256];
  __shared__ uint32_t res[2];
  __shared__ uint32_t bmx[256];
  __shared__ uint32_t bkey[BR_CAP];
  __shared__ int bcol[BR_CAP];
  __shared__ int bsum[4];
  __shared__ uint32_t bres[1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long row = blockIdx.x;
  const int g = (int)(row / B);
  const int k = min(kv[g], n);
  const float* S = reinterpret_cast<const float*>(__builtin_assume_aligned(scores + row * n, 16));
  int* I = idx + row * kmax;
  float* V = val + row * kmax;
  uint32_t key[PL];
#pragma unroll
  for (int i = 0; i < PL / 4; ++i) {
    const int c = (i * 256 + tid) * 4;
    const float4 v = *reinterpret_cast<const float4*>(__builtin_assume_aligned(S + (min(c, n - 4) & ~3), 16));
    const uint32_t live = 0u - (uint32_t)(c < n);
    const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) key[4 * i + j] = order_key(absolute ? fabsf(f[j]) : f[j]) & live;
  }
  bool done = false;
  if (bracket && k > 0 && k <= 256)
    done = bracket_select<PL>(key, k, tid, lane, w, S, I, V, relu, bmx, bkey, bcol, bsum, bres);
  int par = 0;
  auto block_total = [&](int c) {  // one barrier: per-wave DPP totals through parity slots
    c = wave_total(c);
    if (lane == 0) red[par][w] = c;
    __syncthreads();
    const int tot = red[par][0] + red[par][1] + red[par][2] + red[par][3];
    par ^= 1;
    return tot;
  };
  if (k > 0 && !done) {
    uint32_t t = 0;
#pragma unroll 1
    for (int b = 31; b >= LOW; --b) {
      const uint32_t cand = t | (1u << b);
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < PL; ++i) cnt += key[i] >= cand ? 1 : 0;
      if (block_total(cnt) >= k) t = cand;
    }
    const uint32_t hi = t >> LOW;
    int above = 0, inb = 0;
#pragma unroll
    for (int i = 0; i < PL; ++i) {
      const uint32_t h = key[i] >> LOW;
      above += h > hi ? 1 : 0;
      inb += h == hi ? 1 : 0;
    }
    const int n_above = block_total(above);
    const int nb = block_total(inb);
    int gt;
    if (nb <= 64) {
      // compact the bucket (block exclusive scan of the per-thread counts), then wave 0
      // finishes the bisection with ballots
      const int incl = wave_incl_scan(inb, lane);
      if (lane == 63) wsum[par][w] = incl;
      __syncthreads();
      int off = incl - inb;
      for (int ww = 0; ww < w; ++ww) off += wsum[par][ww];
      par ^= 1;
#pragma unroll
      for (int i = 0; i < PL; ++i)
        if ((key[i] >> LOW) == hi) cbuf[off++] = key[i];
      __syncthreads();
      if (w == 0) {
        const bool valid = lane < nb;
        const uint32_t ck = valid ? cbuf[lane] : 0u;
        uint32_t tt = t;
#pragma unroll 1
        for (int b = LOW - 1; b >= 0; --b) {
          const uint32_t cand = tt | (1u << b);
          if (n_above + (int)__popcll(__ballot(valid && ck >= cand)) >= k) tt = cand;
        }
        const int gtv = n_above + (int)__popcll(__ballot(valid && ck > tt));  // all lanes vote
        if (lane == 0) {
          res[0] = tt;
          res[1] = (uint32_t)gtv;
        }
      }
      __syncthreads();
      t = res[0];
      gt = (int)res[1];
    } else {  // crowded bucket: finish by full scans
#pragma unroll 1
      for (int b = LOW - 1; b >= 0; --b) {
        const uint32_t cand = t | (1u << b);
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < PL; ++i) cnt += key[i] >= cand ? 1 : 0;
        if (block_total(cnt) >= k) t = cand;
      }
      int c2 = 0;
#pragma unroll
      for (int i = 0; i < PL; ++i) c2 += key[i] > t ? 1 : 0;
      gt = block_total(c2);
    }
    const int need_ties = k - gt;
    // output in column order: chunk i = columns [1024 i, 1024 i + 1024), thread t owns
    // 4 t .. 4 t + 3 of it; block scans of the tie and take counts give each thread its slots
    int base = 0, ties_seen = 0;
#pragma unroll
    for (int i = 0; i < PL / 4; ++i) {
      int neq = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) neq += key[4 * i + j] == t ? 1 : 0;
      int ie = wave_incl_scan(neq, lane);
      if (lane == 63) wsum[par][w] = ie;
      __syncthreads();
      int tie_rank = ties_seen + ie - neq, tie_tot = 0;
      for (int ww = 0; ww < 4; ++ww) {
        if (ww < w) tie_rank += wsum[par][ww];
        tie_tot += wsum[par][ww];
      }
      par ^= 1;
      bool take[4];
      int ns = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t kk = key[4 * i + j];
        take[j] = kk > t || (kk == t && tie_rank < need_ties);
        tie_rank += kk == t ? 1 : 0;
        ns += take[j] ? 1 : 0;
      }
      int is = wave_incl_scan(ns, lane);
      if (lane == 63) wsum[par][w] = is;
      __syncthreads();
      int pos = base + is - ns, tot = 0;
      for (int ww = 0; ww < 4; ++ww) {
        if (ww < w) pos += wsum[par][ww];
        tot += wsum[par][ww];
      }
      par ^= 1;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (take[j]) {
          const int c = (i * 256 + tid) * 4 + j;
          const float sv = S[c];
          I[pos] = c;
          V[pos] = relu ? fmaxf(sv, 0.f) : sv;
          ++pos;
        }
      }
      base += tot;
      ties_seen += tie_tot;
    }
  }
  for (int j = k + tid; j < kmax; j += 256) {
    I[j] = 0;
    V[j] = 0.f;
  }
}

// ---------------------------------------------------------------------------
// Select on bf16 scores (the scores GEMM's bf16 epilogue: half the bytes of the fp32 score matrix
// written and read).  Keys are the 16-bit orderable bf16 patterns.  bf16 rounding is monotone, so the
// row's k-th largest bf16 key t is the rounding of its k-th largest fp32 score: every key > t belongs
// to the fp32 top-k and every fp32 top-k member has a key >= t -- only the keys EQUAL to t are
// ambiguous.  When they outnumber the slots left (and there are at most TIE_CAP of them), wave 0
// recomputes their exact fp32 scores <x_b, D_hat[g][j]> (the GEMM's bf16 operands, fp32 accumulation)
// and keeps the largest, ties to the lower column.  Kept values are the bf16 scores (after ReLU): the
// precision the codes are stored in downstream.  Same bracket as topk_block_kernel (16-bit bisections);
// more than BR_CAP keys at the bracket (heavy ties, e.g. an all-zero row) fall back to a full
// bisection with ties taken in column order.
__device__ __forceinline__ uint32_t order16(uint32_t h) {
  return (h & 0x8000u) ? (~h & 0xffffu) : (h | 0x8000u);  // larger bf16 -> larger key
}
constexpr int TIE_CAP = 64;

template <int PL>
__device__ __forceinline__ bool bracket_select16(const uint32_t (&key)[PL], int k, int tid, int lane, int w,
                                                 const uint16_t* S, int* I, float* V, int relu, uint32_t* mx,
                                                 uint32_t* ckey, int* ccol, int* wsum, uint32_t* sres, int* tcol,
                                                 float* tsc, int* tkeep, const uint16_t* Xr, const uint16_t* Dg, int d) {
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < PL; ++i) m = max(m, key[i]);
  mx[tid] = m;
  __syncthreads();
  if (w == 0) {
    const uint32_t a0 = mx[lane], a1 = mx[lane + 64], a2 = mx[lane + 128], a3 = mx[lane + 192];
    uint32_t t = 0;
#pragma unroll 1
    for (int b = 15; b >= 0; --b) {
      const uint32_t cand = t | (1u << b);
      const int cnt = __popcll(__ballot(a0 >= cand)) + __popcll(__ballot(a1 >= cand)) +
                      __popcll(__ballot(a2 >= cand)) + __popcll(__ballot(a3 >= cand));
      if (cnt >= k) t = cand;
    }
    if (lane == 0) sres[0] = t;
  }
  __syncthreads();
  const uint32_t lo = sres[0];
  int c = 0;
#pragma unroll
  for (int i = 0; i < PL; ++i) c += key[i] >= lo ? 1 : 0;
  const int incl = wave_incl_scan(c, lane);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int off = incl - c, total = 0;
#pragma unroll
  for (int ww = 0; ww < 4; ++ww) {
    if (ww < w) off += wsum[ww];
    total += wsum[ww];
  }
  if (total > BR_CAP) return false;
#pragma unroll
  for (int i = 0; i < PL / 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (key[8 * i + j] >= lo) {
        ckey[off] = key[8 * i + j];
        ccol[off] = (i * 256 + tid) * 8 + j;
        ++off;
      }
  __syncthreads();
  if (w == 0) {
    const int nq = (total + 63) >> 6;
    uint32_t ck[BR_CAP / 64];
#pragma unroll
    for (int q = 0; q < BR_CAP / 64; ++q) ck[q] = (q < nq && q * 64 + lane < total) ? ckey[q * 64 + lane] : 0u;
    uint32_t t = 0;
#pragma unroll 1
    for (int b = 15; b >= 0; --b) {
      const uint32_t cand = t | (1u << b);
      int cnt = 0;
#pragma unroll
      for (int q = 0; q < BR_CAP / 64; ++q)
        if (q < nq) cnt += __popcll(__ballot(ck[q] >= cand));
      if (cnt >= k) t = cand;
    }
    int gt = 0, nt = 0;
#pragma unroll
    for (int q = 0; q < BR_CAP / 64; ++q)
      if (q < nq) {
        gt += __popcll(__ballot(ck[q] > t));
        nt += __popcll(__ballot(ck[q] == t && q * 64 + lane < total));
      }
    const int need = k - gt;
    // ambiguous ties: exact fp32 scores of the keys equal to t, the `need` largest kept
    const bool exact = Xr && nt > need && nt <= TIE_CAP;
    if (exact) {
      int e0 = 0;
#pragma unroll
      for (int q = 0; q < BR_CAP / 64; ++q)
        if (q < nq) {
          const bool eq = ck[q] == t && q * 64 + lane < total;
          const uint64_t me = __ballot(eq);
          if (eq) tcol[e0 + lanes_below(me)] = ccol[q * 64 + lane];
          e0 += __popcll(me);
        }
      for (int e = 0; e < nt; ++e) {
        const uint16_t* Dr = Dg + (long)tcol[e] * d;
        float dot = 0.f;
        for (int x = lane * 4; x < d; x += 256) {
          const ushort4 a = *reinterpret_cast<const ushort4*>(Xr + x);
          const ushort4 r = *reinterpret_cast<const ushort4*>(Dr + x);
          dot += bf2f(a.x) * bf2f(r.x) + bf2f(a.y) * bf2f(r.y) + bf2f(a.z) * bf2f(r.z) + bf2f(a.w) * bf2f(r.w);
        }
        dot = wave_sum(dot);
        if (lane == 0) tsc[e] = dot;
      }
      if (lane < nt) {
        const float sv = tsc[lane];
        const int cv = tcol[lane];
        int rank = 0;
        for (int e = 0; e < nt; ++e) {
          const float so = tsc[e];
          rank += (so > sv || (so == sv && tcol[e] < cv)) ? 1 : 0;
        }
        tkeep[lane] = rank < need ? 1 : 0;
      }
    }
    int base = 0, ties = 0;
#pragma unroll
    for (int q = 0; q < BR_CAP / 64; ++q) {
      if (q < nq) {
        const uint32_t kk = ck[q];
        const bool eq = kk == t && q * 64 + lane < total;
        const uint64_t me = __ballot(eq);
        const int te = ties + lanes_below(me);
        const bool take = kk > t || (eq && (exact ? tkeep[te] != 0 : te < need));
        const uint64_t mt = __ballot(take);
        if (take) {
          const int pos = base + lanes_below(mt);
          const int col = ccol[q * 64 + lane];
          const float sv = bf2f(S[col]);
          I[pos] = col;
          V[pos] = relu ? fmaxf(sv, 0.f) : sv;
        }
        base += __popcll(mt);
        ties += __popcll(me);
      }
    }
  }
  return true;
}

template <int PL>
__global__ __launch_bounds__(256) void topk_bf16_kernel(const uint16_t* __restrict__ scores, const int* __restrict__ kv,
                                                      int* __restrict__ idx, float* __restrict__ val, int B, int n,
                                                      int kmax, int absolute, int relu, const uint16_t* __restrict__ X,
                                                      long sx, const uint16_t* __restrict__ D, int d) {
  static_assert(PL % 8 == 0, "8 keys per 16-byte load");
  __shared__ int red[2][4];
  __shared__ int wsum[2][4];
  __shared__ uint32_t bmx[256];
  __shared__ uint32_t bkey[BR_CAP];
  __shared__ int bcol[BR_CAP];
  __shared__ int bsum[4];
  __shared__ uint32_t bres[1];
  __shared__ int tcol[TIE_CAP], tkeep[TIE_CAP];
  __shared__ float tsc[TIE_CAP];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = (int)(blockIdx.x % B), g = (int)(blockIdx.x / B);
  const long row = (long)g * B + b;  // scores row [G][B][n]; idx / val are [G][B][kmax]
  const int k = min(kv[g], n);
  const uint16_t* S = scores + row * n;
  int* I = idx + row * kmax;
  float* V = val + row * kmax;
  uint32_t key[PL];
#pragma unroll
  for (int i = 0; i < PL / 8; ++i) {
    const int c = (i * 256 + tid) * 8;
    const uint4 v = *reinterpret_cast<const uint4*>(S + (min(c, n - 8) & ~7));
    const uint32_t live = 0u - (uint32_t)(c < n);
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t h = (wv[j >> 1] >> (16 * (j & 1))) & 0xffffu;
      key[8 * i + j] = order16(absolute ? (h & 0x7fffu) : h) & live;
    }
  }
  const uint16_t* Xr = X ? X + (long)g * sx + (long)b * d : nullptr;
  const uint16_t* Dg = D ? D + (long)g * n * d : nullptr;
  bool done = false;
  if (k > 0 && k <= 256)
    done = bracket_select16<PL>(key, k, tid, lane, w, S, I, V, relu, bmx, bkey, bcol, bsum, bres, tcol, tsc, tkeep,
                                absolute ? nullptr : Xr, Dg, d);
  int par = 0;
  auto block_total = [&](int c) {
    c = wave_total(c);
    if (lane == 0) red[par][w] = c;
    __syncthreads();
    const int tot = red[par][0] + red[par][1] + red[par][2] + red[par][3];
    par ^= 1;
    return tot;
  };
  if (k > 0 && !done) {  // full 16-bit bisection; ties at the threshold in column order
    uint32_t t = 0;
#pragma unroll 1
    for (int bb = 15; bb >= 0; --bb) {
      const uint32_t cand = t | (1u << bb);
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < PL; ++i) cnt += key[i] >= cand ? 1 : 0;
      if (block_total(cnt) >= k) t = cand;
    }
    int c2 = 0;
#pragma unroll
    for (int i = 0; i < PL; ++i) c2 += key[i] > t ? 1 : 0;
    const int need_ties = k - block_total(c2);
    int base = 0, ties_seen = 0;
#pragma unroll
    for (int i = 0; i < PL / 8; ++i) {
      int neq = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) neq += key[8 * i + j] == t ? 1 : 0;
      const int ie = wave_incl_scan(neq, lane);
      if (lane == 63) wsum[par][w] = ie;
      __syncthreads();
      int tie_rank = ties_seen + ie - neq, tie_tot = 0;
      for (int ww = 0; ww < 4; ++ww) {
        if (ww < w) tie_rank += wsum[par][ww];
        tie_tot += wsum[par][ww];
      }
      par ^= 1;
      bool take[8];
      int ns = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t kk = key[8 * i + j];
        take[j] = kk > t || (kk == t && tie_rank < need_ties);
        tie_rank += kk == t ? 1 : 0;
        ns += take[j] ? 1 : 0;
      }
      const int is = wave_incl_scan(ns, lane);
      if (lane == 63) wsum[par][w] = is;
      __syncthreads();
      int pos = base + is - ns, tot = 0;
      for (int ww = 0; ww < 4; ++ww) {
        if (ww < w) pos += wsum[par][ww];
        tot += wsum[par][ww];
      }
      par ^= 1;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (take[j]) {
          const int c = (i * 256 + tid) * 8 + j;
          const float sv = bf2f(S[c]);
          I[pos] = c;
          V[pos] = relu ? fmaxf(sv, 0.f) : sv;
          ++pos;
        }
      }
      base += tot;
      ties_seen += tie_tot;
    }
  }
  for (int j = k + tid; j < kmax; j += 256) {
    I[j] = 0;
    V[j] = 0.f;
  }
}

// One wave per (model, row).  D: [G][n][d] bf16 normalised dictionary (gathered rows).
// Decode gathers the k dictionary rows four at a time (indices and values are
// wave-uniform scalar loads issued ahead of the row loads).  The k code gradients
// <R, D[idx_j]> are reduced sixteen at a time with a butterfly reduce-scatter:
// every lane accumulates 16 partial dots, four exchange steps (8, 4, 2, 1) leave lane
// L with dot j = L & 15 summed over its 16-lane group, two more finish the wave --
// 17 shuffles per 16 dots instead of 6 per dot.
// OCC: minimum waves per SIMD requested from the register allocator (0: compiler's choice);
// DOTS: code gradients reduced per butterfly round (16 rows in flight, or 8 for fewer registers)
// (A/B on config 4, d = 768: 4 waves/SIMD with 16 dots 1.19 ms/step vs 1.32 at the compiler's
// 2 waves; 5-6 waves need 8 dots or spill, and both lose: 1.20-1.23 ms)
template <int NV, int RU = (NV <= 3 ? 8 : 4), int OCC = (NV == 3 ? 4 : 0), int DOTS = 16>
__global__ __launch_bounds__(256, OCC) void topk_decode_grad_kernel(
    const int* __restrict__ idx, const float* __restrict__ val, const int* __restrict__ kv,
    const uint16_t* __restrict__ D, const uint16_t* __restrict__ X, long sx, uint16_t* __restrict__ R,
    float* __restrict__ row_se, uint16_t* __restrict__ codebuf, uint16_t* __restrict__ dscbuf, int G, int B,
    int n, int d, int kmax, float* __restrict__ dscv, const int* __restrict__ prev_idx, int g_dense0) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)G * B) return;
  const int g = row / B, b = row % B;
  const int k = min(kv[g], kmax);
  const int* I = idx + row * kmax;
  const float* V = val + row * kmax;
  const uint16_t* Dg = D + (long)g * n * d;
  float acc[NV * 4];
#pragma unroll
  for (int e = 0; e < NV * 4; ++e) acc[e] = 0.f;
  // loads in flight per lane: NV * RU (more costs occupancy)
  for (int j0 = 0; j0 < k; j0 += RU) {
    int ij[RU];
    float wj[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const bool ok = j0 + u < k;
      ij[u] = ok ? I[j0 + u] : 0;
      wj[u] = ok ? V[j0 + u] : 0.f;  // zero weight: contributes nothing
    }
    // loads are unconditional (clamped column): a guarded load makes hipcc branch and
    // wait vmcnt(0) per load; lanes past d accumulate values that are zeroed below
    ushort4 h[NV][RU];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int e = min((v * 64 + lane) * 4, d - 4);
#pragma unroll
      for (int u = 0; u < RU; ++u) h[v][u] = *reinterpret_cast<const ushort4*>(Dg + (long)ij[u] * d + e);
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        acc[v * 4 + 0] += wj[u] * bf2f(h[v][u].x);
        acc[v * 4 + 1] += wj[u] * bf2f(h[v][u].y);
        acc[v * 4 + 2] += wj[u] * bf2f(h[v][u].z);
        acc[v * 4 + 3] += wj[u] * bf2f(h[v][u].w);
      }
    }
  }
  // residual R = x_hat - x (kept in fp32 registers for the code gradients)
  const uint16_t* Xr = X + (long)g * sx + (long)b * d;
  uint16_t* Rr = R + row * d;
  float se = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int e = (v * 64 + lane) * 4;
    if (e >= d) {  // outside the row: zero so the code-gradient dots below ignore it
      acc[v * 4 + 0] = acc[v * 4 + 1] = acc[v * 4 + 2] = acc[v * 4 + 3] = 0.f;
    } else {
      const ushort4 h = *reinterpret_cast<const ushort4*>(Xr + e);
      acc[v * 4 + 0] -= bf2f(h.x);
      acc[v * 4 + 1] -= bf2f(h.y);
      acc[v * 4 + 2] -= bf2f(h.z);
      acc[v * 4 + 3] -= bf2f(h.w);
      se += acc[v * 4 + 0] * acc[v * 4 + 0] + acc[v * 4 + 1] * acc[v * 4 + 1] +
            acc[v * 4 + 2] * acc[v * 4 + 2] + acc[v * 4 + 3] * acc[v * 4 + 3];
      *reinterpret_cast<ushort4*>(Rr + e) =
          make_ushort4(f2bf(acc[v * 4 + 0]), f2bf(acc[v * 4 + 1]), f2bf(acc[v * 4 + 2]), f2bf(acc[v * 4 + 3]));
    }
  }
  se = wave_sum(se);
  if (lane == 0) row_se[row] = se;
  if (!codebuf) return;
  // models below g_dense0 take the slot-list weight gradient: their dots still feed dscv, but the
  // dense code / code-gradient buffers are never read, so nothing is scattered (or cleared) there
  const bool dense = g >= g_dense0;
  // code gradients (units of R): dscore_j = 1[v_j > 0] <R, D[idx_j]>; scatter code and dscore
  uint16_t* Cb = codebuf + row * (long)n;
  uint16_t* Sb = dscbuf + row * (long)n;
  if (prev_idx && dense) {
    // the previous step's picks of this row go back to zero here (replaces a separate clear
    // launch after the weight gradient); the wait keeps them ordered before the new picks'
    // stores, which may hit the same columns from other lanes of this wave
    const int* P = prev_idx + row * kmax;
    for (int j = lane; j < kmax; j += 64) {
      const int c = P[j];
      Cb[c] = 0;
      Sb[c] = 0;
    }
    __builtin_amdgcn_s_waitcnt(0);
  }
  for (int j0 = 0; j0 < k; j0 += DOTS) {
    float p[DOTS];
#pragma unroll
    for (int u = 0; u < DOTS; ++u) {
      const int j = j0 + u;
      const int ij = j < k ? I[j] : 0;
      const uint16_t* Dr = Dg + (long)ij * d;
      float dot = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int e = min((v * 64 + lane) * 4, d - 4);  // unconditional; acc is 0 past d
        const ushort4 h = *reinterpret_cast<const ushort4*>(Dr + e);
        dot += acc[v * 4 + 0] * bf2f(h.x) + acc[v * 4 + 1] * bf2f(h.y) + acc[v * 4 + 2] * bf2f(h.z) +
               acc[v * 4 + 3] * bf2f(h.w);
      }
      p[u] = dot;
    }
    // butterfly reduce-scatter over lane bits log2(DOTS)-1 .. 0: lane L keeps index L % DOTS
#pragma unroll
    for (int sft = DOTS / 2; sft >= 1; sft >>= 1) {
      const bool upper = (lane & sft) != 0;
#pragma unroll
      for (int t = 0; t < sft; ++t) {
        const float send = upper ? p[t] : p[t + sft];
        const float keep = upper ? p[t + sft] : p[t];
        p[t] = keep + __shfl_xor(send, sft, 64);
      }
    }
    float dot = p[0];
#pragma unroll
    for (int b = DOTS; b < 64; b <<= 1) dot += __shfl_xor(dot, b, 64);
    const int j = j0 + (lane & (DOTS - 1));
    if (lane < DOTS && j < k) {
      const float w = V[j];
      if (w > 0.f && dense) {
        const int c = I[j];
        Cb[c] = f2bf(w);
        Sb[c] = f2bf(dot);
      }
      // per-slot fp32 code gradient for the sparse weight gradient (0 where the code is off)
      if (dscv) dscv[row * kmax + j] = w > 0.f ? dot : 0.f;
    }
  }
}

// ---------------------------------------------------------------------------
// Feature-major slot lists on the device (a counting sort of the picks, no host round trip):
//   slot_count   per (model, block of rows): LDS histogram of the picked features (slots s < k),
//                then one global add per non-empty bin (a popular feature costs one atomic per
//                block, not one per row)
//   slot_offsets per model: exclusive scan of the counts -> list offsets (model bases from k);
//                re-zeroes the counts for the next step
//   slot_scatter per (model, block of rows): reserves each bin's range with one global add, then
//                places the picks with LDS atomics (order within a list is arbitrary here)
//   slot_sort    one wave per list: orders it by batch row -- a 64-lane bitonic sort for short
//                lists, a presence bitmap over the rows for long ones -- so the weight
//                gradient sums in a fixed order (deterministic)
// Slot id = (g B + b) kmax + s: the flat index of the pick in idx / val (and dscv).
__global__ __launch_bounds__(256) void topk_slot_count_kernel(const int* __restrict__ idx, const int* __restrict__ kv,
                                                              int* __restrict__ cnt, int B, int n, int kmax, int rpb) {
  extern __shared__ int hist[];
  const int g = blockIdx.y, b0 = blockIdx.x * rpb, tid = threadIdx.x;
  const int k = min(kv[g], kmax);
  for (int j = tid; j < n; j += 256) hist[j] = 0;
  __syncthreads();
  const int rows = min(rpb, B - b0);
  for (int t = tid; t < rows * k; t += 256) {
    const int r = t / k, sl = t - r * k;
    atomicAdd(&hist[idx[((long)g * B + b0 + r) * kmax + sl]], 1);
  }
  __syncthreads();
  for (int j = tid; j < n; j += 256)
    if (hist[j]) atomicAdd(&cnt[(long)g * n + j], hist[j]);
}

__global__ __launch_bounds__(1024) void topk_slot_offsets_kernel(int* __restrict__ cnt, const int* __restrict__ kv,
                                                                 int* __restrict__ offs, int* __restrict__ cursor,
                                                                 int Gs, int B, int n, int kmax) {
  __shared__ int wsum[16];
  const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  long base = 0;  // slots of the models before g
  for (int q = 0; q < g; ++q) base += (long)B * min(kv[q], kmax);
  const int per = (n + 1023) / 1024;  // consecutive bins per thread
  const int j0 = tid * per;
  int local = 0;
  for (int u = 0; u < per; ++u)
    if (j0 + u < n) local += cnt[(long)g * n + j0 + u];
  // block-wide exclusive scan of the per-thread sums
  int incl = local;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int wbase = 0;
  for (int q = 0; q < w; ++q) wbase += wsum[q];
  int run = (int)base + wbase + incl - local;
  for (int u = 0; u < per; ++u) {
    const int j = j0 + u;
    if (j >= n) break;
    const long r = (long)g * n + j;
    offs[r] = run;
    cursor[r] = run;
    run += cnt[r];
    cnt[r] = 0;  // ready for the next step's counts
  }
  if (g == Gs - 1 && tid == 1023) offs[(long)Gs * n] = run;  // (the last bin's thread holds the end)
}

__global__ __launch_bounds__(256) void topk_slot_scatter_kernel(const int* __restrict__ idx, const int* __restrict__ kv,
                                                                int* __restrict__ cursor, int* __restrict__ tmp, int B,
                                                                int n, int kmax, int rpb) {
  extern __shared__ int lds[];
  int* hist = lds;        // [n] counts, then this block's next position per bin
  const int g = blockIdx.y, b0 = blockIdx.x * rpb, tid = threadIdx.x;
  const int k = min(kv[g], kmax);
  for (int j = tid; j < n; j += 256) hist[j] = 0;
  __syncthreads();
  const int rows = min(rpb, B - b0);
  for (int t = tid; t < rows * k; t += 256) {
    const int r = t / k, sl = t - r * k;
    atomicAdd(&hist[idx[((long)g * B + b0 + r) * kmax + sl]], 1);
  }
  __syncthreads();
  for (int j = tid; j < n; j += 256)
    if (hist[j]) hist[j] = atomicAdd(&cursor[(long)g * n + j], hist[j]);  // reserve this block's range
  __syncthreads();
  for (int t = tid; t < rows * k; t += 256) {
    const int r = t / k, sl = t - r * k;
    const int slot = ((g * B) + b0 + r) * kmax + sl;
    tmp[atomicAdd(&hist[idx[slot]], 1)] = slot;
  }
}

// LB: rows covered by the long-list bitmap path (B <= 64 * LB)
template <int LB>
__global__ __launch_bounds__(256) void topk_slot_sort_kernel(const int* __restrict__ tmp, const int* __restrict__ offs,
                                                             int* __restrict__ perm, long lists, int B, int kmax) {
  __shared__ unsigned long long bits[4][LB];
  __shared__ unsigned char sof[4][64 * LB];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long row = (long)blockIdx.x * 4 + w;
  if (row >= lists) return;
  const int beg = offs[row], L = offs[row + 1] - beg;
  if (L <= 64) {  // bitonic sort of the (unique) slot ids across the wave
    int key = lane < L ? tmp[beg + lane] : 0x7FFFFFFF;
#pragma unroll
    for (int sz = 2; sz <= 64; sz <<= 1)
#pragma unroll
      for (int j = sz >> 1; j > 0; j >>= 1) {
        const int other = __shfl_xor(key, j, 64);
        const bool up = (lane & sz) == 0, low = (lane & j) == 0;
        key = (low == up) ? min(key, other) : max(key, other);
      }
    if (lane < L) perm[beg + lane] = key;
    return;
  }
  // long list: every batch row appears at most once -> presence bitmap over b, then compaction
  // in b order (the slot's s is kept per row)
  const int g_b0 = (tmp[beg] / kmax) / B * B;  // model row base (g B) of this list
  for (int q = lane; q < LB; q += 64) bits[w][q] = 0ull;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  for (int i = lane; i < L; i += 64) {
    const int slot = tmp[beg + i];
    const int gb = slot / kmax, b = gb - g_b0;
    sof[w][b] = (unsigned char)(slot - gb * kmax);
    atomicOr(&bits[w][b >> 6], 1ull << (b & 63));
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  int pos = beg;
  for (int q = 0; q < (B + 63) / 64; ++q) {
    const unsigned long long m = bits[w][q];
    const bool on = (m >> lane) & 1ull;
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (on) {
      const int b = q * 64 + lane;
      perm[pos + before] = (g_b0 + b) * kmax + sof[w][b];
    }
    pos += __popcll(m);
  }
}

// Sparse weight gradient for top-k dictionaries with small k / n (the dense GEMM would multiply
// mostly zeros): for dictionary row j of model g,
//   G[g, j, :] = alpha * sum over the slots (b, s) that picked j of  val * R[g, b, :] + dscv * X[b, :]
// Slot lists come from the device counting sort above, ordered by batch row (deterministic
// summation order).  One wave per dictionary row; rows nobody picked get zeros (Adam reads
// every row).
template <int NV>  // d == 256 * NV
__global__ __launch_bounds__(256) void topk_sparse_wgrad_kernel(const int* __restrict__ perm, const int* __restrict__ offs,
                                                                const float* __restrict__ val,
                                                                const float* __restrict__ dscv,
                                                                const uint16_t* __restrict__ R,
                                                                const uint16_t* __restrict__ X, long sx,
                                                                void* __restrict__ Gout, int Gs, int B, int n, int kmax,
                                                                float alpha, int out_bf16) {
  constexpr int d = NV * 256;
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)Gs * n) return;
  const int g = (int)(row / n);
  const int beg = offs[row], end = offs[row + 1];
  float acc[NV * 4];
#pragma unroll
  for (int e = 0; e < NV * 4; ++e) acc[e] = 0.f;
  for (int e0 = beg; e0 < end; e0 += 2) {  // two slots in flight
    int slot[2];
    float cv[2], sv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool ok = e0 + u < end;
      slot[u] = ok ? perm[e0 + u] : perm[beg];
      cv[u] = ok ? val[slot[u]] : 0.f;
      sv[u] = ok ? dscv[slot[u]] : 0.f;
    }
    ushort4 hr[2][NV], hx[2][NV];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int b = (int)((slot[u] / kmax) % B);
      const uint16_t* Rr = R + ((long)g * B + b) * d;
      const uint16_t* Xr = X + (long)g * sx + (long)b * d;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        hr[u][v] = *reinterpret_cast<const ushort4*>(Rr + (v * 64 + lane) * 4);
        hx[u][v] = *reinterpret_cast<const ushort4*>(Xr + (v * 64 + lane) * 4);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        acc[v * 4 + 0] += cv[u] * bf2f(hr[u][v].x) + sv[u] * bf2f(hx[u][v].x);
        acc[v * 4 + 1] += cv[u] * bf2f(hr[u][v].y) + sv[u] * bf2f(hx[u][v].y);
        acc[v * 4 + 2] += cv[u] * bf2f(hr[u][v].z) + sv[u] * bf2f(hx[u][v].z);
        acc[v * 4 + 3] += cv[u] * bf2f(hr[u][v].w) + sv[u] * bf2f(hx[u][v].w);
      }
  }
  if (out_bf16) {  // the dense weight gradient's bf16 storage (Adam reads one dtype for all models)
    uint16_t* Gr = reinterpret_cast<uint16_t*>(Gout) + row * d;
#pragma unroll
    for (int v = 0; v < NV; ++v)
      *reinterpret_cast<ushort4*>(Gr + (v * 64 + lane) * 4) =
          make_ushort4(f2bf(alpha * acc[v * 4 + 0]), f2bf(alpha * acc[v * 4 + 1]), f2bf(alpha * acc[v * 4 + 2]),
                       f2bf(alpha * acc[v * 4 + 3]));
    return;
  }
  float* Gr = reinterpret_cast<float*>(Gout) + row * d;
#pragma unroll
  for (int v = 0; v < NV; ++v)
    *reinterpret_cast<float4*>(Gr + (v * 64 + lane) * 4) =
        make_float4(alpha * acc[v * 4 + 0], alpha * acc[v * 4 + 1], alpha * acc[v * 4 + 2], alpha * acc[v * 4 + 3]);
}

__global__ __launch_bounds__(256) void topk_clear_kernel(const int* __restrict__ idx, uint16_t* __restrict__ a,
                                                         uint16_t* __restrict__ b, long rows, int n, int kmax) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= rows * kmax) return;
  const long row = t / kmax;
  const int c = idx[t];
  a[row * n + c] = 0;
  b[row * n + c] = 0;
}

// Dense bf16 codes from the select's (idx, val) pairs: codebuf[row, idx] = val for the first
// k[g] slots of each row (the padded slots >= k[g] carry (0, 0.0) and are skipped, so a real
// pick of feature 0 is never overwritten).  For the dense-GEMM decode path.
__global__ __launch_bounds__(256) void topk_scatter_kernel(const int* __restrict__ idx, const float* __restrict__ val,
                                                           const int* __restrict__ kv, uint16_t* __restrict__ code,
                                                           long rows, int rows_per_model, int n, int kmax) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= rows * kmax) return;
  const long row = t / kmax;
  const int s = (int)(t - row * kmax);
  if (s >= kv[row / rows_per_model]) return;
  code[row * n + idx[t]] = f2bf(val[t]);
}


}  // namespace scamd

using namespace scamd;

extern "C" {

int sc_topk_select(const float* scores, const int* k, int* idx, float* val, int G, int B, int n, int kmax,
                   int absolute, int relu, hipStream_t stream) {
  // wave bisection wins up to 64 keys per lane (measured: n = 2048 67 vs 147 us, n = 6144 310 vs 223 us)
  if (n % 4 == 0 && n <= 64 * 64) {
    const long rows = (long)G * B;
    dim3 wgrid((unsigned)((rows + 3) / 4));
#define SC_W(P) \
    if (n <= 64 * P) { hipLaunchKernelGGL((topk_wave_kernel<P>), wgrid, dim3(256), 0, stream, scores, k, idx, val, rows, B, n, \
                                          kmax, absolute, relu); \
      return hipGetLastError() == hipSuccess ? 0 : 3; }
    SC_W(16) SC_W(32) SC_W(64)
#undef SC_W
  }
  if (n % 4 == 0 && n <= 256 * 64) {  // long rows: a block per row
    dim3 bgrid((unsigned)G * B);
    const int bracket = 1;  // bracketed select first (bracket_select; full bisection on heavy ties)
#define SC_BK(P) \
    if (n <= 256 * P) { hipLaunchKernelGGL((topk_block_kernel<P>), bgrid, dim3(256), 0, stream, scores, k, idx, val, B, n, \
                                           kmax, absolute, relu, bracket); \
      return hipGetLastError() == hipSuccess ? 0 : 3; }
    SC_BK(24) SC_BK(32) SC_BK(48) SC_BK(64)
#undef SC_BK
  }
  const int per = (n + 255) / 256;
  dim3 grid((unsigned)G * B);
#define SC_T(P) \
  if (per <= P) { hipLaunchKernelGGL((topk_select_kernel<P>), grid, dim3(256), 0, stream, scores, k, idx, val, B, n, kmax, absolute, relu); \
    return hipGetLastError() == hipSuccess ? 0 : 3; }
  SC_T(4) SC_T(8) SC_T(16) SC_T(24) SC_T(32) SC_T(48) SC_T(64)
#undef SC_T
  return 1;
}

// Per-row top-k of bf16 scores [G][B][n] (see topk_bf16_kernel).  X ([B][d], or [G][B][d] with sx = B d)
// and D ([G][n][d]) are the scores GEMM's bf16 operands, read to resolve ambiguous ties exactly (null:
// ties in column order); absolute = select by |score| (no exact tie resolution).
int sc_topk_select_bf16(const void* scores, const int* k, int* idx, float* val, int G, int B, int n, int kmax,
                        int absolute, int relu, const void* X, long sx, const void* D, int d, hipStream_t stream) {
  if (n % 8 || n < 8 || kmax < 1 || (X && (!D || d % 4 || d < 4))) return 1;
  dim3 grid((unsigned)G * B);
  const uint16_t* S = reinterpret_cast<const uint16_t*>(scores);
  const uint16_t* Xp = reinterpret_cast<const uint16_t*>(X);
  const uint16_t* Dp = reinterpret_cast<const uint16_t*>(D);
#define SC_B16(P) \
  if (n <= 256 * P) { hipLaunchKernelGGL((topk_bf16_kernel<P>), grid, dim3(256), 0, stream, S, k, idx, val, B, n, kmax, \
                                         absolute, relu, Xp, sx, Dp, d); \
    return hipGetLastError() == hipSuccess ? 0 : 3; }
  SC_B16(8) SC_B16(16) SC_B16(24) SC_B16(32) SC_B16(48) SC_B16(64)
#undef SC_B16
  return 1;
}

int sc_topk_decode_grad(const int* idx, const float* val, const int* k, const void* D, const void* X, long sx,
                        void* R, float* row_se, void* codebuf, void* dscbuf, int G, int B, int n, int d, int kmax,
                        hipStream_t stream, float* dscv, const int* prev_idx, int g_dense0) {
  if (d % 4) return 1;
  const int nv = (d + 255) / 256;
  dim3 grid(((long)G * B + 3) / 4);
#define SC_D(V) \
  if (nv <= V) { hipLaunchKernelGGL((topk_decode_grad_kernel<V>), grid, dim3(256), 0, stream, idx, val, k, \
      reinterpret_cast<const uint16_t*>(D), reinterpret_cast<const uint16_t*>(X), sx, reinterpret_cast<uint16_t*>(R), \
      row_se, reinterpret_cast<uint16_t*>(codebuf), reinterpret_cast<uint16_t*>(dscbuf), G, B, n, d, kmax, dscv, prev_idx, \
      g_dense0); \
    return hipGetLastError() == hipSuccess ? 0 : 3; }
  SC_D(1) SC_D(2) SC_D(3) SC_D(4) SC_D(8) SC_D(16)
#undef SC_D
  return 1;
}

// Feature-major slot lists of models [0, Gs): cnt [Gs n] (zero on entry, left zero), offs
// [Gs n + 1], cursor [Gs n], tmp / perm [B sum_g k_g] int32.  Graph-capturable (no host reads).
int sc_topk_slot_lists(const int* idx, const int* k, int* cnt, int* offs, int* cursor, int* tmp, int* perm, int Gs,
                       int B, int n, int kmax, hipStream_t stream) {
  if (n > 32768 || kmax > 256 || Gs < 1 || (long)Gs * B * kmax >= (1l << 31)) return 1;
  const int rpb = 64;
  const dim3 grid((unsigned)((B + rpb - 1) / rpb), (unsigned)Gs);
  const size_t lds = (size_t)n * sizeof(int);
  hipLaunchKernelGGL(topk_slot_count_kernel, grid, dim3(256), lds, stream, idx, k, cnt, B, n, kmax, rpb);
  hipLaunchKernelGGL(topk_slot_offsets_kernel, dim3((unsigned)Gs), dim3(1024), 0, stream, cnt, k, offs, cursor, Gs, B, n,
                     kmax);
  hipLaunchKernelGGL(topk_slot_scatter_kernel, grid, dim3(256), lds, stream, idx, k, cursor, tmp, B, n, kmax, rpb);
  const long lists = (long)Gs * n;
  if (B <= 64 * 32) {
    hipLaunchKernelGGL((topk_slot_sort_kernel<32>), dim3((unsigned)((lists + 3) / 4)), dim3(256), 0, stream, tmp, offs,
                       perm, lists, B, kmax);
  } else if (B <= 64 * 256) {
    hipLaunchKernelGGL((topk_slot_sort_kernel<256>), dim3((unsigned)((lists + 3) / 4)), dim3(256), 0, stream, tmp, offs,
                       perm, lists, B, kmax);
  } else {
    return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// G[0 .. Gs) rows of the weight gradient from the sorted slot lists (see the kernel).
int sc_topk_sparse_wgrad(const int* perm, const int* offs, const float* val, const float* dscv, const void* R,
                         const void* X, long sx, void* Gout, int Gs, int B, int n, int d, int kmax, float alpha,
                         int out_bf16, hipStream_t stream) {
  dim3 grid((unsigned)(((long)Gs * n + 3) / 4));
#define SC_SW(V) \
  if (d == 256 * V) { hipLaunchKernelGGL((topk_sparse_wgrad_kernel<V>), grid, dim3(256), 0, stream, perm, offs, val, dscv, \
      reinterpret_cast<const uint16_t*>(R), reinterpret_cast<const uint16_t*>(X), sx, Gout, Gs, B, n, kmax, alpha, out_bf16); \
    return hipGetLastError() == hipSuccess ? 0 : 3; }
  SC_SW(1) SC_SW(2) SC_SW(3) SC_SW(4)
#undef SC_SW
  return 1;
}

int sc_topk_scatter(const int* idx, const float* val, const int* k, void* code, long rows, int rows_per_model, int n,
                    int kmax, hipStream_t stream) {
  const long total = rows * kmax;
  hipLaunchKernelGGL(topk_scatter_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, idx, val, k,
                     reinterpret_cast<uint16_t*>(code), rows, rows_per_model, n, kmax);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int sc_topk_clear(const int* idx, void* a, void* b, long rows, int n, int kmax, hipStream_t stream) {
  const long total = rows * kmax;
  hipLaunchKernelGGL(topk_clear_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, idx,
                     reinterpret_cast<uint16_t*>(a), reinterpret_cast<uint16_t*>(b), rows, n, kmax);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
