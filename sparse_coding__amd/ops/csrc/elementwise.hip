// Small elementwise kernels of the fused step (gfx950).
//
// center_rows_kernel: the centred per-model input of threshold / learned-centre SAEs,
//   out[g, b, :] = bf16(x[b, :] - c[g, :]),  x bf16 [B, d] shared, c fp32 [G, d]
// in one pass (the torch form was an fp32 [G, B, d] subtraction plus a bf16 copy).
// gather_rows_kernel: the step's batch fetch from the HBM activation ring, out[i] = buf[idx[i]]
//   for 16-byte-multiple rows: one wave per row, every lane one dwordx4 per 1 KiB of the row
//   (the torch index_select took 5.3 us for 2048 x 1 KiB rows, mostly its launch tail).
// lista_fwd_kernel / lista_bwd_kernel: one LISTA layer's elementwise part for a stacked
//   ensemble (reference autoencoders/residual_denoising_autoencoder.py:26-36):
//   r = y + a (a = (x - y D) W^T from the GEMMs), x_ = sign(r) relu(|r| - theta),
//   y' = x_ + m (x_ - xs).  Forward: one pass (the torch chain was ~10 passes over [G, B, n]);
//   backward: one pass producing dr (= dy = da), dxs and per-block partials of dtheta / dm.
#include "common.h"

namespace scamd {

// Optional outputs of the explicit (autograd-free) LISTA step, engine/unrolled.py: r = y + a (may
// alias a: each thread reads its a before writing its r), a bf16 copy of y' (the next GEMM's
// operand), and per-block sums of |y'| (the last layer's L1 term; a block's 1024 elements lie in
// one model because B n % 1024 == 0).
__global__ __launch_bounds__(256) void lista_fwd_kernel(const float4* __restrict__ y, const float4* a,
                                                        const float4* __restrict__ xs, const float* __restrict__ theta,
                                                        const float* __restrict__ m, float4* __restrict__ xo,
                                                        float4* __restrict__ yo, float4* r_out, ushort4* __restrict__ yob,
                                                        float* __restrict__ absp, int B, int n, long total4) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  float ab = 0.f;
  if (t < total4) {
    const long e = t * 4;
    const int g = (int)(e / ((long)B * n));
    const int j = (int)(e % n);
    const float4 yv = y[t], av = a[t], xv = xs[t];
    const float4 th = *reinterpret_cast<const float4*>(theta + (long)g * n + j);
    const float mm = m[g];
    float4 xn, yn, rv;
    auto one = [&](float yy, float aa, float x0, float tt, float& xo_, float& yo_, float& r_) {
      r_ = yy + aa;
      const float mag = fmaxf(fabsf(r_) - tt, 0.f);
      xo_ = r_ > 0.f ? mag : (r_ < 0.f ? -mag : 0.f);
      yo_ = xo_ + mm * (xo_ - x0);
    };
    one(yv.x, av.x, xv.x, th.x, xn.x, yn.x, rv.x);
    one(yv.y, av.y, xv.y, th.y, xn.y, yn.y, rv.y);
    one(yv.z, av.z, xv.z, th.z, xn.z, yn.z, rv.z);
    one(yv.w, av.w, xv.w, th.w, xn.w, yn.w, rv.w);
    xo[t] = xn;
    yo[t] = yn;
    if (r_out) r_out[t] = rv;
    if (yob) yob[t] = make_ushort4(f2bf(yn.x), f2bf(yn.y), f2bf(yn.z), f2bf(yn.w));
    ab = fabsf(yn.x) + fabsf(yn.y) + fabsf(yn.z) + fabsf(yn.w);
  }
  if (absp) {
    __shared__ float red[8];
    ab = block_sum_256(ab, red);
    if (threadIdx.x == 0) absp[blockIdx.x] = ab;
  }
}

// grid (n / 256, B / rb, G), 256 threads = 4 row lanes x 64 column lanes of 4 columns each.
// a == nullptr: y holds r = y + a (the explicit step saves r from the forward).  dL/dy' = gy (+ gy2)
// (+ l1c[g] sign(y'): the last layer's L1 term, y' recomputed).  Outputs, each optional: gr (fp32 dr),
// grb (bf16 gsign * dr), gxs (fp32 dxs); ub = bf16(dr + dxs) for the first layer, whose xs is y itself.
__global__ __launch_bounds__(256) void lista_bwd_kernel(const float* __restrict__ gy, const float* __restrict__ gy2,
                                                        const float* __restrict__ gx, const float* __restrict__ y,
                                                        const float* __restrict__ a, const float* __restrict__ xs,
                                                        const float* __restrict__ theta, const float* __restrict__ m,
                                                        const float* __restrict__ l1c, float* __restrict__ gr,
                                                        uint16_t* __restrict__ grb, float gsign, float* __restrict__ gxs,
                                                        uint16_t* __restrict__ ub, float* __restrict__ gth_part,
                                                        float* __restrict__ gm_part, int B, int n, int rb) {
  __shared__ float4 red4[4][64];
  __shared__ float redm[256];
  const int g = blockIdx.z, rbk = blockIdx.y;
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int j = blockIdx.x * 256 + cl * 4;
  const float mm = m[g];
  const float lc = l1c ? l1c[g] : 0.f;
  const float4 th = *reinterpret_cast<const float4*>(theta + (long)g * n + j);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 gt = z4;
  float gmv = 0.f;
  for (int r = rbk * rb + rl; r < (rbk + 1) * rb; r += 4) {
    const long o = ((long)g * B + r) * n + j;
    const float4 gyv = *reinterpret_cast<const float4*>(gy + o);
    const float4 gy2v = gy2 ? *reinterpret_cast<const float4*>(gy2 + o) : z4;
    const float4 gxv = gx ? *reinterpret_cast<const float4*>(gx + o) : z4;
    const float4 yv = *reinterpret_cast<const float4*>(y + o);
    const float4 av = a ? *reinterpret_cast<const float4*>(a + o) : z4;
    const float4 xv = *reinterpret_cast<const float4*>(xs + o);
    float4 gro, gxo;
    auto one = [&](float gyy, float gyy2, float gxx, float yy, float aa, float x0, float tt, float& gro_, float& gxo_,
                   float& gtt) {
      const float r_ = yy + aa;
      const float mag = fabsf(r_) - tt;
      const float on = mag > 0.f ? 1.f : 0.f;
      const float sg = r_ > 0.f ? 1.f : (r_ < 0.f ? -1.f : 0.f);
      const float xo_ = sg * fmaxf(mag, 0.f);
      float gyt = gyy + gyy2;
      if (l1c) {
        const float yo_ = xo_ + mm * (xo_ - x0);
        gyt += lc * (yo_ > 0.f ? 1.f : (yo_ < 0.f ? -1.f : 0.f));
      }
      const float gtot = (1.f + mm) * gyt + gxx;   // dL/dx_
      gro_ = gtot * on * (sg != 0.f ? 1.f : 0.f);  // d x_/d r = 1 where |r| > theta (0 at r = 0)
      gxo_ = -mm * gyt;
      gtt -= gtot * sg * on;                        // d x_/d theta = -sign(r) where |r| > theta
      gmv += gyt * (xo_ - x0);                      // d y'/d m = x_ - xs
    };
    one(gyv.x, gy2v.x, gxv.x, yv.x, av.x, xv.x, th.x, gro.x, gxo.x, gt.x);
    one(gyv.y, gy2v.y, gxv.y, yv.y, av.y, xv.y, th.y, gro.y, gxo.y, gt.y);
    one(gyv.z, gy2v.z, gxv.z, yv.z, av.z, xv.z, th.z, gro.z, gxo.z, gt.z);
    one(gyv.w, gy2v.w, gxv.w, yv.w, av.w, xv.w, th.w, gro.w, gxo.w, gt.w);
    if (gr) *reinterpret_cast<float4*>(gr + o) = gro;
    if (gxs) *reinterpret_cast<float4*>(gxs + o) = gxo;
    if (grb)
      *reinterpret_cast<ushort4*>(grb + o) =
          make_ushort4(f2bf(gsign * gro.x), f2bf(gsign * gro.y), f2bf(gsign * gro.z), f2bf(gsign * gro.w));
    if (ub)
      *reinterpret_cast<ushort4*>(ub + o) = make_ushort4(f2bf(gro.x + gxo.x), f2bf(gro.y + gxo.y),
                                                         f2bf(gro.z + gxo.z), f2bf(gro.w + gxo.w));
  }
  red4[rl][cl] = gt;
  redm[threadIdx.x] = gmv;
  __syncthreads();
  if (rl == 0) {
    float4 s = red4[0][cl];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      s.x += red4[k][cl].x; s.y += red4[k][cl].y; s.z += red4[k][cl].z; s.w += red4[k][cl].w;
    }
    *reinterpret_cast<float4*>(gth_part + ((long)g * gridDim.y + rbk) * n + j) = s;
  }
  for (int w = 128; w > 0; w >>= 1) {
    __syncthreads();
    if (threadIdx.x < w) redm[threadIdx.x] += redm[threadIdx.x + w];
  }
  if (threadIdx.x == 0) gm_part[((long)g * gridDim.y + rbk) * gridDim.x + blockIdx.x] = redm[0];
}

// Residual-denoising layers, explicit step (reference autoencoders/residual_denoising_autoencoder.py:
// 92-122: c' = relu(c + theta) W^T + c, codes relu(c_L + b)).  res_fwd: c' = u + c (u = the layer GEMM,
// absent for the first layer: c' = c), written to cout when given; hb = bf16(relu(c' + th)) with th the
// NEXT layer's theta; `fin`: th is the encoder bias, cout = relu(c' + b) (the codes), hb their bf16
// copy and absp the |c| block sums (B n % 1024 == 0).
__global__ __launch_bounds__(256) void res_fwd_kernel(const float4* __restrict__ u, const float4* __restrict__ c,
                                                      const float* __restrict__ th, float4* __restrict__ cout,
                                                      ushort4* __restrict__ hb, float* __restrict__ absp, int fin,
                                                      int B, int n, long total4) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  float ab = 0.f;
  if (t < total4) {
    const long e = t * 4;
    const int g = (int)(e / ((long)B * n));
    const int j = (int)(e % n);
    float4 cv = c[t];
    if (u) {
      const float4 uv = u[t];
      cv.x += uv.x; cv.y += uv.y; cv.z += uv.z; cv.w += uv.w;
    }
    const float4 tv = *reinterpret_cast<const float4*>(th + (long)g * n + j);
    const float4 h = make_float4(fmaxf(cv.x + tv.x, 0.f), fmaxf(cv.y + tv.y, 0.f), fmaxf(cv.z + tv.z, 0.f),
                                 fmaxf(cv.w + tv.w, 0.f));
    if (fin) {
      cout[t] = h;
      ab = h.x + h.y + h.z + h.w;
    } else if (cout) {
      cout[t] = cv;
    }
    hb[t] = make_ushort4(f2bf(h.x), f2bf(h.y), f2bf(h.z), f2bf(h.w));
  }
  if (absp) {
    __shared__ float red[8];
    ab = block_sum_256(ab, red);
    if (threadIdx.x == 0) absp[blockIdx.x] = ab;
  }
}

// res_bwd, grid (n / 256, B / rb, G): m = 1[pre + th > 0] (th optional); t = gadd, or gin + l1c[g]
// without gadd; out = (gadd ? gin : 0) + t m (fp32 optional) and outb = bf16(out); cpart[G][B / rb][n]
// = column sums of t m (the layer's theta gradient, or with the codes as `pre` the bias gradient).
__global__ __launch_bounds__(256) void res_bwd_kernel(const float* __restrict__ gin, const float* __restrict__ gadd,
                                                      const float* __restrict__ pre, const float* __restrict__ th,
                                                      const float* __restrict__ l1c, float* __restrict__ out,
                                                      uint16_t* __restrict__ outb, float* __restrict__ cpart, int B,
                                                      int n, int rb) {
  __shared__ float4 red4[4][64];
  const int g = blockIdx.z, rbk = blockIdx.y;
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int j = blockIdx.x * 256 + cl * 4;
  const float lc = l1c ? l1c[g] : 0.f;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 tv = th ? *reinterpret_cast<const float4*>(th + (long)g * n + j) : z4;
  float4 cs = z4;
  for (int r = rbk * rb + rl; r < (rbk + 1) * rb; r += 4) {
    const long o = ((long)g * B + r) * n + j;
    const float4 gi = *reinterpret_cast<const float4*>(gin + o);
    const float4 pv = *reinterpret_cast<const float4*>(pre + o);
    float4 tt;
    if (gadd) tt = *reinterpret_cast<const float4*>(gadd + o);
    else tt = make_float4(gi.x + lc, gi.y + lc, gi.z + lc, gi.w + lc);
    const float4 mt = make_float4(pv.x + tv.x > 0.f ? tt.x : 0.f, pv.y + tv.y > 0.f ? tt.y : 0.f,
                                  pv.z + tv.z > 0.f ? tt.z : 0.f, pv.w + tv.w > 0.f ? tt.w : 0.f);
    float4 ov = mt;
    if (gadd) {
      ov.x += gi.x; ov.y += gi.y; ov.z += gi.z; ov.w += gi.w;
    }
    if (out) *reinterpret_cast<float4*>(out + o) = ov;
    *reinterpret_cast<ushort4*>(outb + o) = make_ushort4(f2bf(ov.x), f2bf(ov.y), f2bf(ov.z), f2bf(ov.w));
    cs.x += mt.x; cs.y += mt.y; cs.z += mt.z; cs.w += mt.w;
  }
  red4[rl][cl] = cs;
  __syncthreads();
  if (rl == 0) {
    float4 s = red4[0][cl];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      s.x += red4[k][cl].x; s.y += red4[k][cl].y; s.z += red4[k][cl].z; s.w += red4[k][cl].w;
    }
    *reinterpret_cast<float4*>(cpart + ((long)g * gridDim.y + rbk) * n + j) = s;
  }
}

__global__ __launch_bounds__(256) void center_rows_kernel(const uint16_t* __restrict__ x, const float* __restrict__ c,
                                                          uint16_t* __restrict__ out, int G, int B, int d) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;  // one thread per 4 elements of out
  const long per_model = (long)B * d / 4;
  if (t >= (long)G * per_model) return;
  const int g = (int)(t / per_model);
  const long e = (t - (long)g * per_model) * 4;  // element offset inside [B, d]
  const int k = (int)(e % d);
  const ushort4 xv = *reinterpret_cast<const ushort4*>(x + e);
  const float4 cv = *reinterpret_cast<const float4*>(c + (long)g * d + k);
  *reinterpret_cast<ushort4*>(out + (long)g * B * d + e) =
      make_ushort4(f2bf(bf2f(xv.x) - cv.x), f2bf(bf2f(xv.y) - cv.y), f2bf(bf2f(xv.z) - cv.z), f2bf(bf2f(xv.w) - cv.w));
}

__global__ __launch_bounds__(256) void gather_rows_kernel(const u32x4_t* __restrict__ buf, const long* __restrict__ idx,
                                                          u32x4_t* __restrict__ out, long rows, int row_vec) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63;
  const long src = idx[r];
  const u32x4_t* s = buf + src * row_vec;
  u32x4_t* o = out + r * row_vec;
  for (int v = lane; v < row_vec; v += 64) o[v] = s[v];
}

// gather_rows_perm_kernel: the same fetch with the indices taken from a ring permutation at a
//   DEVICE cursor, (step - epoch_start) * rows, so the batch fetch can live inside the step's
//   HIP graph (the engine's device step counter advances in the graph; the host only rolls a
//   new permutation between replays at epoch ends).  Out-of-range positions read row 0.
__global__ __launch_bounds__(256) void gather_rows_perm_kernel(const u32x4_t* __restrict__ buf, long nbuf,
                                                               const long* __restrict__ perm, long nperm,
                                                               const int* __restrict__ step,
                                                               const int* __restrict__ ep0,
                                                               u32x4_t* __restrict__ out, long rows, int row_vec,
                                                               long stride, long offset, long inner, long ostride) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63;
  // (data parallel: stride = N B, offset = rank B -- this rank's shard of each global batch;
  // several steps at once: `inner` rows per step, step k of the group at perm block +k stride and
  // at output row k ostride -- e.g. straight into this rank's slot of each step's global batch)
  const long k = r / inner, i = r - k * inner;
  const long j = (long)(step[0] - ep0[0]) * stride + offset + k * stride + i;
  long src = (j >= 0 && j < nperm) ? perm[j] : 0;
  src = (src >= 0 && src < nbuf) ? src : 0;
  const u32x4_t* s = buf + src * row_vec;
  u32x4_t* o = out + (k * ostride + i) * row_vec;
  for (int v = lane; v < row_vec; v += 64) o[v] = s[v];
}

// gather_rows_blocks_kernel: out[o * inner + i] = buf[perm[base + o * stride + i]] -- several
//   steps' shards of a data-parallel permutation in one launch (rank r of N, step t: the block at
//   perm[(t N + r) B, +B)), so a multi-step group's local batches fill one send buffer.
//   Out-of-range positions read row 0.
__global__ __launch_bounds__(256) void gather_rows_blocks_kernel(const u32x4_t* __restrict__ buf, long nbuf,
                                                                 const long* __restrict__ perm, long nperm, long base,
                                                                 long stride, long inner, u32x4_t* __restrict__ out,
                                                                 long rows, int row_vec) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63;
  const long o = r / inner;
  const long j = base + o * stride + (r - o * inner);
  long src = (j >= 0 && j < nperm) ? perm[j] : 0;
  src = (src >= 0 && src < nbuf) ? src : 0;
  const u32x4_t* s = buf + src * row_vec;
  u32x4_t* dst = out + r * row_vec;
  for (int v = lane; v < row_vec; v += 64) dst[v] = s[v];
}

}  // namespace scamd

using namespace scamd;

extern "C" {

int sc_center_rows(const void* x, const float* c, void* out, int G, int B, int d, hipStream_t stream) {
  if (d % 4 || G < 1 || B < 1) return 1;
  const long total = (long)G * B * d / 4;
  hipLaunchKernelGGL(center_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream,
                     reinterpret_cast<const uint16_t*>(x), c, reinterpret_cast<uint16_t*>(out), G, B, d);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int sc_lista_fwd(const float* y, const float* a, const float* xs, const float* theta, const float* m, float* xo,
                 float* yo, int G, int B, int n, hipStream_t stream) {
  if (n % 4 || G < 1 || B < 1) return 1;
  const long total4 = (long)G * B * n / 4;
  hipLaunchKernelGGL(lista_fwd_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, stream,
                     reinterpret_cast<const float4*>(y), reinterpret_cast<const float4*>(a),
                     reinterpret_cast<const float4*>(xs), theta, m, reinterpret_cast<float4*>(xo),
                     reinterpret_cast<float4*>(yo), nullptr, nullptr, nullptr, B, n, total4);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// The explicit step's forward: also r (may be a itself), the bf16 y', and |y'| block sums
// absp[G][B n / 1024] (needs B n % 1024 == 0).
int sc_lista_fwd2(const float* y, const float* a, const float* xs, const float* theta, const float* m, float* xo,
                  float* yo, float* r_out, void* yob, float* absp, int G, int B, int n, hipStream_t stream) {
  if (n % 4 || G < 1 || B < 1 || (absp && ((long)B * n) % 1024)) return 1;
  const long total4 = (long)G * B * n / 4;
  hipLaunchKernelGGL(lista_fwd_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, stream,
                     reinterpret_cast<const float4*>(y), reinterpret_cast<const float4*>(a),
                     reinterpret_cast<const float4*>(xs), theta, m, reinterpret_cast<float4*>(xo),
                     reinterpret_cast<float4*>(yo), reinterpret_cast<float4*>(r_out),
                     reinterpret_cast<ushort4*>(yob), absp, B, n, total4);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// gth_part: [G][B / rb][n], gm_part: [G][B / rb][n / 256]
int sc_lista_bwd(const float* gy, const float* gx, const float* y, const float* a, const float* xs,
                 const float* theta, const float* m, float* gr, float* gxs, float* gth_part, float* gm_part,
                 int G, int B, int n, int rb, hipStream_t stream) {
  if (n % 256 || rb < 4 || rb % 4 || B % rb || G < 1) return 1;
  hipLaunchKernelGGL(lista_bwd_kernel, dim3(n / 256, B / rb, G), dim3(256), 0, stream, gy, nullptr, gx, y, a, xs,
                     theta, m, nullptr, gr, nullptr, 1.f, gxs, nullptr, gth_part, gm_part, B, n, rb);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int sc_lista_bwd2(const float* gy, const float* gy2, const float* gx, const float* y, const float* a, const float* xs,
                  const float* theta, const float* m, const float* l1c, float* gr, void* grb, float gsign, float* gxs,
                  void* ub, float* gth_part, float* gm_part, int G, int B, int n, int rb, hipStream_t stream) {
  if (n % 256 || rb < 4 || rb % 4 || B % rb || G < 1) return 1;
  hipLaunchKernelGGL(lista_bwd_kernel, dim3(n / 256, B / rb, G), dim3(256), 0, stream, gy, gy2, gx, y, a, xs,
                     theta, m, l1c, gr, reinterpret_cast<uint16_t*>(grb), gsign, gxs, reinterpret_cast<uint16_t*>(ub),
                     gth_part, gm_part, B, n, rb);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int sc_res_fwd(const float* u, const float* c, const float* th, float* cout, void* hb, float* absp, int fin, int G,
               int B, int n, hipStream_t stream) {
  if (n % 4 || G < 1 || B < 1 || (absp && ((long)B * n) % 1024) || (fin && !cout)) return 1;
  const long total4 = (long)G * B * n / 4;
  hipLaunchKernelGGL(res_fwd_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, stream,
                     reinterpret_cast<const float4*>(u), reinterpret_cast<const float4*>(c), th,
                     reinterpret_cast<float4*>(cout), reinterpret_cast<ushort4*>(hb), absp, fin, B, n, total4);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int sc_res_bwd(const float* gin, const float* gadd, const float* pre, const float* th, const float* l1c, float* out,
               void* outb, float* cpart, int G, int B, int n, int rb, hipStream_t stream) {
  if (n % 256 || rb < 4 || rb % 4 || B % rb || G < 1) return 1;
  hipLaunchKernelGGL(res_bwd_kernel, dim3(n / 256, B / rb, G), dim3(256), 0, stream, gin, gadd, pre, th, l1c, out,
                     reinterpret_cast<uint16_t*>(outb), cpart, B, n, rb);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int sc_gather_rows(const void* buf, const long* idx, void* out, long rows, long row_bytes, hipStream_t stream) {
  if (row_bytes % 16 || rows < 0) return 1;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream,
                     reinterpret_cast<const u32x4_t*>(buf), idx, reinterpret_cast<u32x4_t*>(out), rows,
                     (int)(row_bytes / 16));
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int sc_gather_rows_perm(const void* buf, long nbuf, const long* perm, long nperm, const int* step, const int* ep0,
                        void* out, long rows, long row_bytes, long stride, long offset, long inner, long ostride,
                        hipStream_t stream) {
  if (inner <= 0) inner = rows;
  if (ostride <= 0) ostride = inner;
  if (row_bytes % 16 || rows < 0 || nbuf < 1 || stride < inner || offset < 0 || rows % inner || ostride < inner)
    return 1;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(gather_rows_perm_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream,
                     reinterpret_cast<const u32x4_t*>(buf), nbuf, perm, nperm, step, ep0,
                     reinterpret_cast<u32x4_t*>(out), rows, (int)(row_bytes / 16), stride, offset, inner, ostride);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int sc_gather_rows_blocks(const void* buf, long nbuf, const long* perm, long nperm, long base, long stride,
                          long inner, long outer, void* out, long row_bytes, hipStream_t stream) {
  if (row_bytes % 16 || inner < 1 || outer < 0 || nbuf < 1) return 1;
  const long rows = inner * outer;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(gather_rows_blocks_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream,
                     reinterpret_cast<const u32x4_t*>(buf), nbuf, perm, nperm, base, stride, inner,
                     reinterpret_cast<u32x4_t*>(out), rows, (int)(row_bytes / 16));
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
